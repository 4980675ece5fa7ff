"""Multi-GPU plan of the secagg path (fedbiomed_amd/distributed.py).

CPU (gloo, world_size 2, 127.0.0.1): the party-per-rank exchange -- LOM reduce-scatter of
masked u64 sums, JL all-to-all of ciphertext stripes, all-gather of float64 stripes --
composed with the CPU oracle as the per-rank compute, must reproduce the single-process
oracle result bit for bit.  GPU: the same exchange with the HIP kernels as every rank's
compute (2 gloo ranks sharing cuda:0, spawned before any GPU initialisation), and
element-range shards computed with global offsets (elem_offset / ct_offset) concatenate to
the unsharded device result.
"""

import os
import socket

import numpy as np
import pytest
import torch

from fedbiomed_amd import distributed as Dd
from fedbiomed_amd import workload as W
from oracle import secagg_oracle as O

P, TAU = 4, 3


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn_name, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, globals()[fn_name](rank, world)))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, e))
    finally:
        dist.destroy_process_group()


def _spawn(fn_name, world=2):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, v = q.get(timeout=240)
        out[r] = v
    for p in procs:
        p.join(timeout=60)
    for r, v in out.items():
        if isinstance(v, Exception):
            raise v
    return out


# ---- per-rank bodies (module level: spawn pickles them by name) --------------------------
N_LOM = 1003  # ragged: not a multiple of 8 * world


def _lom_party_per_rank(rank, world):
    ids = W.node_ids(P)
    nonce = O.lom_nonce(W.LOM_NONCE)
    mine = [p for p in range(P) if p % world == rank]
    ys = [O.lom_encrypt([float(v) for v in W.party_params(p, N_LOM)], TAU, ids[p],
                        W.pairwise_secrets_for(ids[p], ids), ids, nonce, weight=W.party_weight(p)) for p in mine]
    local = torch.from_numpy(O.lom_aggregate(ys).view(np.int64).copy())
    stripe = Dd.reduce_scatter_u64(local, N_LOM)
    sums = [int(v) for v in stripe.numpy().view(np.uint64)]
    total_w = sum(W.party_weight(p) for p in range(P))
    out = torch.from_numpy(np.asarray(O.reverse_quantize(O.apply_average(sums, total_w)), dtype=np.float64))
    return Dd.all_gather_stripes(out, N_LOM, 8).numpy()


N_JL = 100


def _jl_party_per_rank(rank, world):
    from fedbiomed_amd import _device as D

    keys = [W.jl_user_key(p) for p in range(P)]
    mine = [p for p in range(P) if (p // (P // world)) == rank]  # rank-major party blocks
    cts = [O.jl_encrypt([float(v) for v in W.party_params(p, N_JL)], TAU, keys[p], W.BIPRIME0, P,
                        weight=W.party_weight(p)) for p in mine]
    limbs = torch.from_numpy(np.stack([D.ints_to_limbs(c) for c in cts]).view(np.int32).copy())
    stripe, k0 = Dd.all_to_all_ciphertexts(limbs, P // world)
    es, cr = O.jl_slot(None, P)
    e_lo, e_hi = min(k0 * cr, N_JL), min((k0 + stripe.shape[1]) * cr, N_JL)
    ints = [D.limbs_to_ints(stripe[u].numpy()) for u in range(P)]
    total_w = sum(W.party_weight(p) for p in range(P))
    out = O.jl_crypter_aggregate(ints, TAU, -sum(keys), W.BIPRIME0, total_w, e_hi - e_lo, k0=k0)
    out = torch.from_numpy(np.asarray(out, dtype=np.float64))
    return Dd.all_gather_stripes(out, N_JL, cr).numpy(), (e_lo, e_hi)


# ---- per-rank bodies with the HIP path as each rank's compute (cuda:0 shared by the ranks) ----
N_LOM_HIP = 100_003  # ragged: not a multiple of 8 * world
N_JL_HIP = 3_001


def _lom_party_per_rank_hip(rank, world):
    """LOM: HIP protect of this rank's parties -> HIP column sum (mod 2^64) -> reduce-scatter
    of the masked sums -> HIP average + dequantise of the rank's stripe -> all-gather
    (reference LOM.aggregate _lom.py:177-192 + _secagg_crypter.py:394-455)."""
    from fedbiomed_amd import _device as D
    from fedbiomed_amd.secagg import SecaggLomCrypter

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ids = W.node_ids(P)
    lc = SecaggLomCrypter(W.LOM_NONCE)
    mine = [p for p in range(P) if p % world == rank]
    Y = torch.stack([lc.encrypt_tensor(TAU, ids[p], torch.from_numpy(W.party_params(p, N_LOM_HIP)).to(dev),
                                       W.pairwise_secrets_for(ids[p], ids), ids, weight=W.party_weight(p))
                     for p in mine])
    _, local = D.lom_aggregate(Y, 1, want_out=False, want_sums=True)
    stripe = Dd.reduce_scatter_u64(local.cpu(), N_LOM_HIP)  # gloo: host tensors
    total_w = sum(W.party_weight(p) for p in range(P))
    out = lc.aggregate_tensor(stripe.view(1, -1).to(dev), total_w)
    return Dd.all_gather_stripes(out.cpu(), N_LOM_HIP, 8).numpy()


def _jl_party_per_rank_hip(rank, world):
    """JL: HIP encrypt of this rank's parties -> all-to-all of ciphertext stripes -> HIP
    aggregate of the rank's stripe with its global ct_offset -> all-gather (reference
    _jls.py:646-699, product :691-693)."""
    from fedbiomed_amd.secagg import SecaggCrypter

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    keys = [W.jl_user_key(p) for p in range(P)]
    jc = SecaggCrypter()
    mine = [p for p in range(P) if (p // (P // world)) == rank]
    cts = torch.stack([jc.encrypt_tensor(P, TAU, torch.from_numpy(W.party_params(p, N_JL_HIP)).to(dev), keys[p],
                                         W.BIPRIME0, weight=W.party_weight(p)) for p in mine]).cpu()
    stripe, k0 = Dd.all_to_all_ciphertexts(cts, P // world)
    es, cr = O.jl_slot(None, P)
    e_lo, e_hi = min(k0 * cr, N_JL_HIP), min((k0 + stripe.shape[1]) * cr, N_JL_HIP)
    total_w = sum(W.party_weight(p) for p in range(P))
    out = jc.aggregate_tensor(TAU, stripe.to(dev), -sum(keys), W.BIPRIME0, total_w, num_expected_params=e_hi - e_lo,
                              ct_offset=k0)
    return Dd.all_gather_stripes(out.cpu(), N_JL_HIP, cr).numpy(), (e_lo, e_hi)


def _gather_shards(rank, world):
    """Each rank holds its shard_range stripe of a known vector; the gather rebuilds it whole."""
    res = []
    for n, align in ((1003, 8), (10_001, 30), (5, 8)):
        lo, hi = Dd.shard_range(n, world, rank, align)
        full = torch.arange(n, dtype=torch.float64) * 0.5 - 3.0
        res.append(Dd.all_gather_shards(full[lo:hi].clone(), n, align).numpy())
    return res


N8_U64 = 10_003  # ragged: not a multiple of 8 * 8
N8_CT = 1_237  # ciphertexts per party, ragged over 8 stripes


def _local_u64(rank):
    """Rank r's local masked sum: deterministic int64 bit patterns spanning the whole u64 range."""
    rng = np.random.default_rng(800 + rank)
    return rng.integers(-2**63, 2**63 - 1, N8_U64, dtype=np.int64, endpoint=True)


def _local_cts(rank, ppr):
    """Rank r's parties' ciphertext limbs [ppr, N8_CT, 64] (int32), distinct per (party, ct, limb)."""
    rng = np.random.default_rng(900 + rank)
    return rng.integers(-2**31, 2**31 - 1, (ppr, N8_CT, 64), dtype=np.int32, endpoint=True)


def _world8_collectives(rank, world):
    """every collective of distributed.py at the driver's world size -- the LOM
    reduce-scatter of u64 sums, the stripes' all-gather back, the JL all-to-all of ciphertext stripes
    (one and two parties per rank) and the element-range split's final gather -- on gloo."""
    out = {}
    stripe = Dd.reduce_scatter_u64(torch.from_numpy(_local_u64(rank)), N8_U64)
    out["rs_stripe"] = stripe.numpy().copy()
    out["rs_full"] = Dd.all_gather_stripes(stripe, N8_U64, 8).numpy()
    for ppr in (1, 2):
        got, k0 = Dd.all_to_all_ciphertexts(torch.from_numpy(_local_cts(rank, ppr)), ppr)
        out[f"a2a{ppr}"] = (got.numpy(), k0)
    lo, hi = Dd.shard_range(10_000_000, world, rank, 30)
    full = torch.arange(lo, hi, dtype=torch.float64) * 0.25
    g = Dd.all_gather_shards(full, 10_000_000, 30)
    out["shards_ok"] = bool(torch.equal(g, torch.arange(10_000_000, dtype=torch.float64) * 0.25))
    return out


def test_world8_collectives_equal_single_rank_gloo():
    """The 8-rank form of every exchange (gloo, 8 processes, 127.0.0.1) equals the single-rank
    result: the u64 sum mod 2^64 of all ranks' vectors, every party's ciphertexts in rank-major party
    order for each stripe of stripe_bounds, and the whole output vector on every rank."""
    world = 8
    res = _spawn("_world8_collectives", world)
    with np.errstate(over="ignore"):
        want = sum(_local_u64(r).view(np.uint64) for r in range(world)).view(np.int64)
    per, bounds = Dd.stripe_bounds(N8_U64, world, 8)
    cper, cbounds = Dd.stripe_bounds(N8_CT, world, 1)
    for r in range(world):
        lo, hi = bounds[r]
        assert np.array_equal(res[r]["rs_stripe"], want[lo:hi]), r
        assert np.array_equal(res[r]["rs_full"], want), r
        for ppr in (1, 2):
            allp = np.concatenate([_local_cts(q, ppr) for q in range(world)])  # rank-major parties
            got, k0 = res[r][f"a2a{ppr}"]
            c0, c1 = cbounds[r]
            assert k0 == c0 and np.array_equal(got, allp[:, c0:c1]), (r, ppr)
        assert res[r]["shards_ok"], r


# ---- tests ---------------------------------------------------------------------------------
@pytest.mark.parametrize("world", [2, 3])
def test_all_gather_shards_gloo(world):
    """The bench's final gather of the element-range output stripes (uneven shard_range stripes)."""
    res = _spawn("_gather_shards", world)
    for r in range(world):
        for n, got in zip((1003, 10_001, 5), res[r]):
            assert got.tolist() == (np.arange(n, dtype=np.float64) * 0.5 - 3.0).tolist()


@pytest.mark.parametrize("n,world,align", [(0, 2, 8), (7, 2, 8), (1003, 2, 8), (10_000_000, 8, 8),
                                           (10_000_000, 8, 30), (100, 3, 31)])
def test_shard_range_tiles(n, world, align):
    prev = 0
    for r in range(world):
        lo, hi = Dd.shard_range(n, world, r, align)
        assert lo == prev and lo <= hi and (lo % align == 0 or lo == n)
        prev = hi
    assert prev == n
    per, bounds = Dd.stripe_bounds(n, world, align)
    assert per % align == 0 and bounds[-1][1] == n and all(b[0] % align == 0 or b[0] == n for b in bounds)


def test_lom_party_per_rank_gloo():
    res = _spawn("_lom_party_per_rank")
    ids = W.node_ids(P)
    nonce = O.lom_nonce(W.LOM_NONCE)
    ys = [O.lom_encrypt([float(v) for v in W.party_params(p, N_LOM)], TAU, ids[p], W.pairwise_secrets_for(ids[p], ids),
                        ids, nonce, weight=W.party_weight(p)) for p in range(P)]
    ref = O.lom_crypter_aggregate(ys, sum(W.party_weight(p) for p in range(P)))
    for r in range(2):
        assert res[r].view(np.uint64).tolist() == np.asarray(ref, dtype=np.float64).view(np.uint64).tolist()


def test_jl_party_per_rank_gloo():
    res = _spawn("_jl_party_per_rank")
    keys = [W.jl_user_key(p) for p in range(P)]
    cts = [O.jl_encrypt([float(v) for v in W.party_params(p, N_JL)], TAU, keys[p], W.BIPRIME0, P,
                        weight=W.party_weight(p)) for p in range(P)]
    ref = O.jl_crypter_aggregate(cts, TAU, -sum(keys), W.BIPRIME0, sum(W.party_weight(p) for p in range(P)), N_JL)
    assert res[0][1][0] == 0 and res[1][1][1] == N_JL and res[0][1][1] == res[1][1][0]
    for r in range(2):
        assert res[r][0].view(np.uint64).tolist() == np.asarray(ref, dtype=np.float64).view(np.uint64).tolist()


def test_jl_stripe_oracle_offsets():
    """The oracle's k0 stripes concatenate to the whole-vector ciphertexts (CPU)."""
    keys = W.jl_user_key(0)
    x = [float(v) for v in W.party_params(0, 200)]
    es, cr = O.jl_slot(None, 4)
    whole = O.jl_encrypt(x, TAU, keys, W.BIPRIME0, 4)
    lo, hi = Dd.jl_shard(200, 2, 1, cr)
    part = O.jl_encrypt(x[lo:hi], TAU, keys, W.BIPRIME0, 4, k0=lo // cr)
    assert part == whole[lo // cr:]


# ---- GPU: sharded offsets reproduce the unsharded device result ------------------------------
@pytest.mark.gpu
def test_lom_elem_offset_shards_gpu():
    from fedbiomed_amd.secagg import SecaggLomCrypter

    dev = torch.device("cuda", 0)
    n, world = 100_003, 3
    ids = W.node_ids(3)
    x = torch.from_numpy(W.party_params(1, n)).to(dev)
    lc = SecaggLomCrypter(W.LOM_NONCE)
    sec = W.pairwise_secrets_for(ids[1], ids)
    whole = lc.encrypt_tensor(TAU, ids[1], x, sec, ids, weight=77)
    parts = []
    for r in range(world):
        lo, hi = Dd.lom_shard(n, world, r)
        parts.append(lc.encrypt_tensor(TAU, ids[1], x[lo:hi], sec, ids, weight=77, elem_offset=lo))
    assert torch.equal(torch.cat(parts), whole)


@pytest.mark.gpu
def test_jl_ct_offset_shards_gpu():
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = torch.device("cuda", 0)
    n, world, Pp = 5_000, 3, 3
    keys = [W.jl_user_key(p) for p in range(Pp)]
    xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(Pp)]
    jc = SecaggCrypter()
    es, cr = O.jl_slot(None, Pp)
    whole = torch.stack([jc.encrypt_tensor(Pp, TAU, xs[p], keys[p], W.BIPRIME0, weight=10 + p) for p in range(Pp)])
    out_whole = jc.aggregate_tensor(TAU, whole, -sum(keys), W.BIPRIME0, 33, num_expected_params=n)
    outs = []
    for r in range(world):
        lo, hi = Dd.jl_shard(n, world, r, cr)
        cts = torch.stack([jc.encrypt_tensor(Pp, TAU, xs[p][lo:hi], keys[p], W.BIPRIME0, weight=10 + p,
                                             ct_offset=lo // cr) for p in range(Pp)])
        assert torch.equal(cts, whole[:, lo // cr:(hi + cr - 1) // cr])
        outs.append(jc.aggregate_tensor(TAU, cts, -sum(keys), W.BIPRIME0, 33, num_expected_params=hi - lo,
                                        ct_offset=lo // cr))
    assert torch.equal(torch.cat(outs), out_whole)


@pytest.mark.gpu
def test_lom_party_per_rank_hip_gloo():
    res = _spawn("_lom_party_per_rank_hip")
    ids = W.node_ids(P)
    nonce = O.lom_nonce(W.LOM_NONCE)
    ys = [O.lom_encrypt(W.party_params(p, N_LOM_HIP).astype(np.float64), TAU, ids[p],
                        W.pairwise_secrets_for(ids[p], ids), ids, nonce, weight=W.party_weight(p)) for p in range(P)]
    ref = O.lom_crypter_aggregate(ys, sum(W.party_weight(p) for p in range(P)))
    for r in range(2):
        assert res[r].view(np.uint64).tolist() == np.asarray(ref, dtype=np.float64).view(np.uint64).tolist()


@pytest.mark.gpu
def test_jl_party_per_rank_hip_gloo():
    res = _spawn("_jl_party_per_rank_hip")
    keys = [W.jl_user_key(p) for p in range(P)]
    cts = [O.jl_encrypt([float(v) for v in W.party_params(p, N_JL_HIP)], TAU, keys[p], W.BIPRIME0, P,
                        weight=W.party_weight(p)) for p in range(P)]
    ref = O.jl_crypter_aggregate(cts, TAU, -sum(keys), W.BIPRIME0, sum(W.party_weight(p) for p in range(P)),
                                 N_JL_HIP)
    assert res[0][1][0] == 0 and res[1][1][1] == N_JL_HIP and res[0][1][1] == res[1][1][0]
    for r in range(2):
        assert res[r][0].view(np.uint64).tolist() == np.asarray(ref, dtype=np.float64).view(np.uint64).tolist()


# ---- the RCCL branches: a world-1 "nccl" group on cuda:0 (one GPU per box) -----------------
def _collectives_world1_body():
    """Every collective of distributed.py on device tensors (int64, float64, int32) plus the LOM
    party-per-rank exchange with HIP compute, in a world-1 group of the spawning backend."""
    from fedbiomed_amd import _device as D
    from fedbiomed_amd.secagg import SecaggLomCrypter

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    local = torch.randint(-2**62, 2**62, (1003,), dtype=torch.int64, generator=g).to(dev)
    f64 = torch.randn(1003, dtype=torch.float64, generator=g).to(dev)
    cts = torch.randint(-2**31, 2**31 - 1, (2, 37, 64), dtype=torch.int32, generator=g).to(dev)
    out = {
        "reduce_scatter_u64": Dd.reduce_scatter_u64(local, 1003).cpu(),
        "all_gather_stripes": Dd.all_gather_stripes(f64, 1003, 8).cpu(),
        "all_gather_shards_f64": Dd.all_gather_shards(f64, 1003, 30).cpu(),
        "all_gather_shards_i32": Dd.all_gather_shards(cts[0, :, 0].contiguous(), 37, 1).cpu(),
    }
    stripe, k0 = Dd.all_to_all_ciphertexts(cts, 2)
    out["all_to_all_ciphertexts"] = stripe.cpu()
    out["k0"] = k0
    out["inputs"] = (local.cpu(), f64.cpu(), cts.cpu())
    # the LOM party-per-rank leg: HIP protect -> HIP u64 column sum -> reduce-scatter -> HIP average
    ids = W.node_ids(P)
    lc = SecaggLomCrypter(W.LOM_NONCE)
    Y = torch.stack([lc.encrypt_tensor(TAU, ids[p], torch.from_numpy(W.party_params(p, N_LOM)).to(dev),
                                       W.pairwise_secrets_for(ids[p], ids), ids, weight=W.party_weight(p))
                     for p in range(P)])
    _, sums = D.lom_aggregate(Y, 1, want_out=False, want_sums=True)
    red = Dd.reduce_scatter_u64(sums, N_LOM)
    agg = lc.aggregate_tensor(red.view(1, -1), sum(W.party_weight(p) for p in range(P)))
    out["lom_pp"] = Dd.all_gather_stripes(agg, N_LOM, 8).cpu()
    torch.cuda.synchronize()
    # numpy, not tensors: torch's queue shares tensors through file descriptors that die with
    # the child process
    return {k: (tuple(t.numpy() for t in v) if isinstance(v, tuple) else v.numpy() if isinstance(v, torch.Tensor)
                else v) for k, v in out.items()}


def _world1_worker(backend, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    try:
        torch.cuda.set_device(0)
        dist.init_process_group(backend, rank=0, world_size=1)
        try:
            q.put((dist.get_backend(), _collectives_world1_body()))
        finally:
            dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((backend, e))


def _run_world1(backend):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world1_worker, args=(backend, _free_port(), q))
    p.start()
    got_backend, res = q.get(timeout=240)
    p.join(timeout=60)
    if isinstance(res, Exception):
        raise res
    assert got_backend == backend
    return res


@pytest.mark.gpu
def test_rccl_collectives_world1():
    """The "nccl" (= RCCL) branches of distributed.py -- reduce_scatter_tensor, all_gather_into_tensor,
    all_to_all_single -- run once on the GPU (a world-1 group in a fresh spawned process, before any
    GPU call), equal to the gloo branches on the same inputs and to the collectives' meaning at world
    size 1; the LOM party-per-rank exchange with HIP compute through them equals the oracle
    (reference LOM.aggregate, _lom.py:177-192)."""
    nccl, gloo = _run_world1("nccl"), _run_world1("gloo")

    def same(a, b):
        return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))

    for k in ("reduce_scatter_u64", "all_gather_stripes", "all_gather_shards_f64", "all_gather_shards_i32",
              "all_to_all_ciphertexts", "lom_pp"):
        assert same(nccl[k], gloo[k]), k
    local, f64, cts = nccl["inputs"]
    assert same(nccl["reduce_scatter_u64"], local)
    assert same(nccl["all_gather_stripes"], f64) and same(nccl["all_gather_shards_f64"], f64)
    assert same(nccl["all_gather_shards_i32"], np.ascontiguousarray(cts[0, :, 0]))
    assert nccl["k0"] == 0 and same(nccl["all_to_all_ciphertexts"], cts)
    ids = W.node_ids(P)
    nonce = O.lom_nonce(W.LOM_NONCE)
    ys = [O.lom_encrypt(W.party_params(p, N_LOM).astype(np.float64), TAU, ids[p], W.pairwise_secrets_for(ids[p], ids),
                        ids, nonce, weight=W.party_weight(p)) for p in range(P)]
    ref = O.lom_crypter_aggregate(ys, sum(W.party_weight(p) for p in range(P)))
    assert nccl["lom_pp"].view(np.uint64).tolist() == np.asarray(ref, np.float64).view(np.uint64).tolist()
