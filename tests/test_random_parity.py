"""Randomised parity sweep: the HIP path through the reference API against the CPU oracle on
seeded random configurations -- party counts, lengths (incl. 1 and ragged), rounds up to
2^64-1, weights, clipping/target ranges (training and the federated-analytics 10^14 / 2^55
range), user keys of either sign, special floats (NaN, +-inf, -0.0, beyond the clipping
range).  Bit-exact: integers compared exactly, float64 outputs as bit patterns; where the
oracle raises (LOM overflow guard), the device path must raise too."""

import numpy as np
import pytest

from fedbiomed_amd import workload as W
from fedbiomed_amd.constants import SAParameters
from oracle import secagg_oracle as O

pytestmark = pytest.mark.gpu

SPECIAL = [float("nan"), float("inf"), -float("inf"), -0.0, 0.0, 1e300, -1e300, 2.5, -2.5]


def _params(rng, n, clip):
    x = rng.standard_normal(n) * (clip if clip else 3) * 0.6
    k = int(rng.integers(0, min(n, 6) + 1))
    for i in rng.choice(n, k, replace=False):
        x[i] = SPECIAL[int(rng.integers(0, len(SPECIAL)))]
    return [float(v) for v in x]


def _ranges(rng):
    choice = int(rng.integers(0, 5))
    return [(None, None), (1, 2**10), (7, 2**20), (3, 2**13), (10**14, 2**55)][choice]


def _bits(xs):
    return np.asarray(xs, dtype=np.float64).view(np.uint64).tolist()


@pytest.fixture(scope="module")
def dev():
    from fedbiomed_amd import _device as D

    return D.device()


@pytest.mark.parametrize("seed", range(12))
def test_lom_random(dev, seed):
    from fedbiomed_amd.exceptions import FedbiomedSecaggError
    from fedbiomed_amd.secagg import SecaggLomCrypter

    rng = np.random.default_rng(100 + seed)
    P = int(rng.integers(2, 10))
    n = int(rng.choice([1, 7, 8, 9, int(rng.integers(2, 400))]))
    tau = int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2)) if seed % 3 == 0 else int(rng.integers(0, 50))
    clip, target = _ranges(rng)
    nonce_str = "".join(chr(int(c)) for c in rng.integers(48, 123, size=int(rng.integers(1, 20))))
    ids = sorted(f"node-{int(v):04x}" for v in rng.choice(2**16, P, replace=False))
    ws = [int(rng.integers(1, 2**16)) for _ in range(P)]
    xs = [_params(rng, n, clip) for _ in range(P)]
    cr = SecaggLomCrypter(nonce_str)
    nonce = O.lom_nonce(nonce_str)
    ys = []
    for p, u in enumerate(ids):
        sec = W.pairwise_secrets_for(u, ids)
        try:
            ref = [int(v) for v in O.lom_encrypt(xs[p], tau, u, sec, ids, nonce, clip=clip, weight=ws[p],
                                                 target=target)]
        except O.OracleError as e:
            assert "FB417" in str(e)
            with pytest.raises(FedbiomedSecaggError):
                cr.encrypt(tau, u, xs[p], sec, ids, clipping_range=clip, weight=ws[p], target_range=target)
            return
        got = cr.encrypt(tau, u, xs[p], sec, ids, clipping_range=clip, weight=ws[p], target_range=target)
        assert got == ref, (seed, p)
        ys.append(got)
    total = sum(ws)
    out = cr.aggregate(ys, total, clipping_range=clip, target_range=target)
    assert _bits(out) == _bits(O.lom_crypter_aggregate(ys, total, clip=clip, target=target))


@pytest.mark.parametrize("seed", range(8))
def test_jl_random(dev, seed):
    from fedbiomed_amd.secagg import SecaggCrypter

    rng = np.random.default_rng(200 + seed)
    P = int(rng.integers(2, 7))
    clip, target = _ranges(rng)
    es, cr_ = O.jl_slot(target, P)
    n = int(rng.choice([1, cr_, cr_ + 1, int(rng.integers(2, 4 * cr_))]))
    tau = int(rng.integers(0, 2**63)) * 2 + 1 if seed % 2 else int(rng.integers(0, 100))
    ws = [int(rng.integers(1, 2**16)) for _ in range(P)]
    keys = [(-1 if rng.integers(0, 2) else 1) * W.jl_user_key(50 + 10 * seed + p) for p in range(P)]
    xs = [_params(rng, n, clip) for _ in range(P)]
    jc = SecaggCrypter()
    cts = []
    for p in range(P):
        got = jc.encrypt(P, tau, xs[p], keys[p], W.BIPRIME0, clipping_range=clip, weight=ws[p],
                         target_range=target)
        assert got == O.jl_encrypt(xs[p], tau, keys[p], W.BIPRIME0, P, clip=clip, weight=ws[p], target=target), p
        cts.append(got)
    sk0 = -sum(keys)
    n_exp = int(rng.integers(1, n + 2))
    out = jc.aggregate(tau, P, cts, sk0, W.BIPRIME0, sum(ws), clipping_range=clip, num_expected_params=n_exp,
                       target_range=target)
    ref = O.jl_crypter_aggregate(cts, tau, sk0, W.BIPRIME0, sum(ws), n_exp, clip=clip, target=target)
    assert _bits(out) == _bits(ref)


@pytest.mark.parametrize("bits", [2, 5, 17, 64, 300, 511, 1000, 1023, 1024])
def test_jl_random_moduli(dev, bits):
    """The N-adic exponentiation engine on random odd moduli of every size class (its digit
    bounds scale with N / 2^1036; small moduli hit FDH retries, i.e. wide digests): raw
    UserKey.encrypt of int64 plaintexts with keys of either sign and several lengths, and the
    server decrypt of the party product, against the oracle's closed forms."""
    import random

    import torch

    from fedbiomed_amd import _device as D

    rng = random.Random(1000 + bits)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    if N < 3:
        N = 3
    n, P, tau = 37, 3, rng.getrandbits(64)
    pts = [rng.getrandbits(63) for _ in range(n)]
    keys = [rng.getrandbits(rng.choice([1, 40, 700, 2040])) * rng.choice([1, -1]) for _ in range(P)]
    if bits in (17, 1024):
        keys[1] = 0  # key 0: H^0 = 1 (the engine's key_is_zero path), c = N*pt + 1
    x = torch.tensor(pts, dtype=torch.int64, device=dev)
    cts = []
    for key in keys:
        got = D.jl_encrypt(x, N, key, tau, P, slot=(100, 1))
        ints = D.limbs_to_ints(got.cpu().numpy())
        n2 = N * N
        want = [((N * pt + 1) % n2) * O.powmod(O.fdh((k << 512) | tau, n2), key, n2) % n2
                for k, pt in enumerate(pts)]
        assert ints == want, (bits, key)
        cts.append(got)
    sk0 = -sum(keys)
    _, sums = D.jl_aggregate(torch.stack(cts), N, sk0, tau, n, 1, want_out=False, want_sums=True, slot=(100, 1))
    s = sums.cpu().numpy().view(np.uint64)
    got = [int(a) | (int(b) << 64) for a, b in s]
    n2 = N * N
    want = []
    for k in range(n):
        prod = 1
        for c in cts:
            prod = prod * D.limbs_to_ints(c[k:k + 1].cpu().numpy())[0] % n2
        v = prod * O.powmod(O.fdh((k << 512) | tau, n2), sk0, n2) % n2
        want.append(((v - 1) // N) % N)
    assert got == want, bits


@pytest.mark.parametrize("P", [16, 17, 31, 33])
def test_jl_many_parties(dev, P):
    """Party counts past the bench's 8: the slot width grows with ceil(log2(P + 1))
    (es = 35 at P = 16, 17 and 31; 36 at P = 33 -- `_jls.py:104-116`), so the ciphertext
    count per vector changes; encrypt and the P-way ciphertext product bit-exact."""
    from fedbiomed_amd.secagg import SecaggCrypter

    rng = np.random.default_rng(300 + P)
    es, cr_ = O.jl_slot(None, P)
    assert es == 30 + int(np.ceil(np.log2(P + 1)))
    n = 2 * cr_ + 3
    tau = int(rng.integers(0, 2**40))
    ws = [int(rng.integers(1, 2**16)) for _ in range(P)]
    keys = [W.jl_user_key(900 + p) for p in range(P)]
    xs = [_params(rng, n, None) for _ in range(P)]
    jc = SecaggCrypter()
    cts = []
    for p in range(P):
        got = jc.encrypt(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p])
        if p in (0, P - 1):
            assert got == O.jl_encrypt(xs[p], tau, keys[p], W.BIPRIME0, P, weight=ws[p]), p
        cts.append(got)
    out = jc.aggregate(tau, P, cts, -sum(keys), W.BIPRIME0, sum(ws), num_expected_params=n)
    ref = O.jl_crypter_aggregate(cts, tau, -sum(keys), W.BIPRIME0, sum(ws), n)
    assert _bits(out) == _bits(ref)


@pytest.mark.parametrize("seed", range(16))
def test_jl_random_tensor_engines(dev, seed):
    """The device-tensor path on random configurations under each exponentiation engine (one
    lane, quad, triple, auto policy), half of them with the parties' exponentiations in one
    batched launch: sampled ciphertexts against the oracle's UserKey.encrypt, the decoded
    integer sums exact for every element, and the float64 outputs bit-exact."""
    import torch

    from fedbiomed_amd import _device as D
    from fedbiomed_amd.secagg import SecaggCrypter

    rng = np.random.default_rng(500 + seed)
    P = int(rng.integers(2, 13))
    clip, target = _ranges(rng)
    es, cr_ = O.jl_slot(target, P)
    n = int(rng.choice([1, cr_, cr_ + 1, int(rng.integers(2, 40_000))]))
    tau = int(rng.integers(0, 2**63)) * 2 + 1 if seed % 3 == 0 else int(rng.integers(0, 100))
    ws = [int(rng.integers(1, 2**16)) for _ in range(P)]
    keys = [int(rng.choice([-1, 1])) * W.jl_user_key(300 + 20 * seed + p) for p in range(P)]
    if seed % 5 == 0:
        keys[0] = 0
    engine = ("single", "quad", "triple", "auto")[seed % 4]
    batch = seed % 2 == 1
    xs = [np.asarray(_params(rng, n, clip), dtype=np.float64) for _ in range(P)]
    xd = [torch.tensor(x, dtype=torch.float64, device=dev) for x in xs]
    jc = SecaggCrypter()
    sk0 = -sum(keys)
    kw = dict(clipping_range=clip, target_range=target)
    with D.jl_engine(engine):
        if batch:
            with D.deferred_checks():
                pend = [jc.encrypt_tensor(P, tau, xd[p], keys[p], W.BIPRIME0, weight=ws[p], defer_exp=True, **kw)
                        for p in range(P)]
                with D.jl_exp_batch(dev):
                    cts = [q.finish() for q in pend]
        else:
            cts = [jc.encrypt_tensor(P, tau, xd[p], keys[p], W.BIPRIME0, weight=ws[p], **kw) for p in range(P)]
        C = torch.stack(cts)
        out, sums = jc.aggregate_tensor(tau, C, sk0, W.BIPRIME0, sum(ws), num_expected_params=n, want_sums=True,
                                        **kw)
    n_ct = C.shape[1]
    tr = target or O.TARGET_RANGE
    qw = [[int(v) * ws[p] for v in O.quantize(xs[p], clip, tr)] for p in range(P)]
    ks = sorted({0, n_ct - 1, *rng.choice(n_ct, min(n_ct, 4), replace=False).tolist()})
    for p in range(P):
        got = D.limbs_to_ints(C[p, ks].cpu().numpy())
        for k, g in zip(ks, got):
            assert g == O.jl_encrypt_ints(qw[p][k * cr_:(k + 1) * cr_], tau, keys[p], W.BIPRIME0, P,
                                          target=target, k0=k)[0], (seed, p, k)
    want = [sum(col) for col in zip(*qw)]
    s = sums.cpu().numpy().view(np.uint64)
    assert [int(a) | (int(b) << 64) for a, b in s] == want, seed
    ref = O.reverse_quantize(O.apply_average(want, sum(ws)), clip, tr)
    assert _bits(out.cpu().numpy()) == _bits(ref)


@pytest.mark.parametrize("n_ct", [255, 256, 257, 512])
def test_jl_aggregate_block_boundaries(dev, n_ct):
    """Ciphertext counts around the 256-lane workgroups of the combine (jl_prod_kernel: operand
    column in LDS) and of the factor's inverse lift (jl_lift_kernel: output rows staged through
    LDS, a partial last workgroup writes only its own rows): outputs bit-exact vs the oracle."""
    from fedbiomed_amd.secagg import SecaggCrypter

    rng = np.random.default_rng(7000 + n_ct)
    P, clip, target = 3, 3, SAParameters.TARGET_RANGE
    es, cr_ = O.jl_slot(target, P)
    n = n_ct * cr_ - int(rng.integers(0, cr_))
    keys = [W.jl_user_key(900 + p) for p in range(P)]
    xs = [_params(rng, n, clip) for _ in range(P)]
    jc = SecaggCrypter()
    cts = [jc.encrypt(P, 5, xs[p], keys[p], W.BIPRIME0, clipping_range=clip) for p in range(P)]
    assert len(cts[0]) == n_ct
    out = jc.aggregate(5, P, cts, -sum(keys), W.BIPRIME0, P, clipping_range=clip, num_expected_params=n)
    ref = O.jl_crypter_aggregate(cts, 5, -sum(keys), W.BIPRIME0, P, n, clip=clip)
    assert _bits(out) == _bits(ref)


def test_lom_more_peers_than_one_argument_block(dev):
    """70 parties: every node has 69 peers, past the 64-peer kernel-argument block (the first group
    with the quantise / overflow statistics, the rest accumulated in place): masked vectors
    bit-exact vs the oracle for a few nodes, and all 70 masks cancel in the aggregate."""
    from fedbiomed_amd.secagg import LOM

    rng = np.random.default_rng(70)
    ids = [f"n{u:03d}" for u in range(70)]
    n, tau, nonce = 37, 12345, bytes(range(16))
    xs = [rng.integers(0, 2**20, size=n).tolist() for _ in ids]
    ys = [LOM(nonce=nonce).protect(u, W.pairwise_secrets_for(u, ids), tau, xs[p], ids) for p, u in enumerate(ids)]
    for p in (0, 33, 69):
        ref = O.lom_protect(ids[p], W.pairwise_secrets_for(ids[p], ids), tau, xs[p], ids, nonce)
        assert ys[p] == [int(v) for v in ref]
    assert LOM(nonce=nonce).aggregate(ys) == [sum(c) for c in zip(*xs)]
