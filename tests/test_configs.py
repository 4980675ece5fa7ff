"""BASELINE.json configurations as GPU parity cases, at their own sizes.

  cfg 1  LOM mask+unmask, 1k elements, 2 parties             -> bit-exact vs the oracle, whole vector
  cfg 2  JL encrypt+aggregate, 100k elements, 4 parties        -> sampled ciphertexts bit-exact vs the
                                                                  oracle + exact decoded sums (all elements)
  cfg 3  LOM round of the 101 notebook's MNIST net, 4 nodes    -> one party bit-exact, mask cancellation
         (1,199,882 parameters)                     exact over all elements
  cfg 4  JL encrypt+aggregate, 10M elements, 8 parties,       -> the 8 ct_offset stripes of an 8-GPU
         element-range sharded across 8 GPUs                     split concatenate bit-exactly to the
                                                                  whole vector, sampled ciphertexts bit-
                                                                  exact vs the oracle, decoded sums exact
                                                                  over all 10M elements, stripe aggregates
                                                                  == whole aggregate, sampled float64
                                                                  outputs bit-exact
  cfg 5  LOM masking + additive secret sharing, 100M elements, -> mask cancellation exact, sampled
         16 parties                                               windows bit-exact, split/reconstruct exact
Oracle = oracle/secagg_oracle.py (pinned to the reference's own
vectors in tests/test_oracle_golden.py).  Tolerance: 0 -- integers compared exactly, float64
outputs compared as bit patterns.
"""

import numpy as np
import pytest
import torch

from fedbiomed_amd import _device as D, workload as W
from oracle import secagg_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return D.device()


def _u64(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def _qw(x: np.ndarray, w: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        return O.quantize(x) * np.uint64(w)


def _oracle_outputs(want: np.ndarray, total_w: int) -> np.ndarray:
    """The reference's float64 outputs for every element: reverse_quantize(_apply_average(sums)) of the
    oracle's exact integer sums.  _apply_average is Python's int / int (correctly rounded); for sums and
    weights below 2^53 both convert to float64 exactly and IEEE division rounds the same quotient, so numpy
    gives it for the whole vector -- pinned against the oracle's own apply_average on a sample."""
    assert int(want.max()) < 2**53 and total_w < 2**53
    avg = want.astype(np.float64) / float(total_w)
    idx = np.linspace(0, len(want) - 1, 4096).astype(np.int64)
    assert avg[idx].tolist() == O.apply_average([int(v) for v in want[idx]], total_w)
    c = O.CLIPPING_RANGE  # reverse_quantize (_secagg_utils.py:152-187): truncate to u64, then -c + step * u
    step = (c - (-c)) / (O.TARGET_RANGE - 1)
    out = float(-c) + step * avg.astype(np.uint64).astype(np.float64)
    assert out[idx].view(np.uint64).tolist() == O.reverse_quantize(avg[idx].tolist()).view(np.uint64).tolist()
    return out


def _lom_window_oracle(u, ids, tau, qw_window, offset, nonce):
    """LOM.protect (secagg/_lom.py:105-175) restricted to elements [offset, offset+len):
    ChaCha20 blocks from offset/8 on (the keystream is counter-indexed)."""
    n = len(qw_window)
    mask = np.zeros(n, dtype=np.uint64)
    idx = (np.arange(offset, offset + n, dtype=np.uint64) + np.uint64(tau)).byteswap()
    sec = W.pairwise_secrets_for(u, ids)
    with np.errstate(over="ignore"):
        for p in ids:
            if p == u:
                continue
            seed = O.prf_eval_key(sec[p], nonce, tau)
            ks = O.chacha20_blocks(seed, nonce, offset // 8, (n + 7) // 8).astype("<u4").view("<u8").reshape(-1)[:n]
            vec = ks ^ idx
            mask = mask + vec if p < u else mask - vec
        return mask + qw_window


def test_cfg1_lom_1k_2_parties(dev):
    from fedbiomed_amd.secagg import SecaggLomCrypter

    n, P, tau = 1000, 2, 1
    ids, ws = W.node_ids(P), [W.party_weight(p) for p in range(P)]
    cr = SecaggLomCrypter(W.LOM_NONCE)
    xs = [W.party_params(p, n).astype(np.float64).tolist() for p in range(P)]
    ys = [cr.encrypt(tau, u, xs[p], W.pairwise_secrets_for(u, ids), ids, weight=ws[p]) for p, u in enumerate(ids)]
    for p, u in enumerate(ids):
        ref = O.lom_encrypt(xs[p], tau, u, W.pairwise_secrets_for(u, ids), ids, O.lom_nonce(W.LOM_NONCE),
                            weight=ws[p])
        assert ys[p] == [int(v) for v in ref]
    out = cr.aggregate(ys, sum(ws))
    assert np.array_equal(np.asarray(out).view(np.uint64), O.lom_crypter_aggregate(ys, sum(ws)).view(np.uint64))


def test_cfg2_jl_100k_4_parties(dev):
    from fedbiomed_amd.secagg import SecaggCrypter

    n, P, tau = 100_000, 4, 1
    ws = [W.party_weight(p) for p in range(P)]
    keys = [W.jl_user_key(p) for p in range(P)]
    es, cr_ = O.jl_slot(None, P)
    jc = SecaggCrypter()
    xs = [W.party_params(p, n) for p in range(P)]
    cts = torch.stack([jc.encrypt_tensor(P, tau, torch.from_numpy(xs[p]).to(dev), keys[p], W.BIPRIME0, weight=ws[p])
                       for p in range(P)])
    n_ct = (n + cr_ - 1) // cr_
    assert tuple(cts.shape) == (P, n_ct, 64)
    # sampled ciphertexts (first, last/partial, random) bit-exact vs the oracle
    rng = np.random.default_rng(2)
    ks = sorted({0, n_ct - 1, *rng.choice(n_ct, 24, replace=False).tolist()})
    for p in range(P):
        qw = [int(v) for v in _qw(xs[p], ws[p])]
        got = D.limbs_to_ints(cts[p, ks].cpu().numpy())
        for k, g in zip(ks, got):
            ref = O.jl_encrypt_ints(qw[k * cr_:(k + 1) * cr_], tau, keys[p], W.BIPRIME0, P, k0=k)[0]
            assert g == ref, (p, k)
    # aggregate: the decoded integer sums are exactly sum_p q_p w_p for every element
    out, sums = jc.aggregate_tensor(tau, cts, -sum(keys), W.BIPRIME0, sum(ws), num_expected_params=n,
                                    want_sums=True)
    sums = sums.cpu().numpy().view(np.uint64).reshape(n, 2)
    want = np.zeros(n, dtype=np.uint64)
    for p in range(P):
        want += _qw(xs[p], ws[p])
    assert (sums[:, 1] == 0).all() and np.array_equal(sums[:, 0], want)
    ref = O.reverse_quantize(O.apply_average([int(v) for v in want], sum(ws)))
    assert np.array_equal(out.cpu().numpy().view(np.uint64), ref.view(np.uint64))


def test_cfg3_lom_mnist_round_4_nodes(dev):
    from fedbiomed_amd.secagg import SecaggLomCrypter

    n, P, tau = 1_199_882, 4, 3
    ids, ws = W.node_ids(P), [W.party_weight(p) for p in range(P)]
    nonce = O.lom_nonce(W.LOM_NONCE)
    cr = SecaggLomCrypter(W.LOM_NONCE)
    xs = [W.party_params(p, n) for p in range(P)]
    Y = torch.stack([cr.encrypt_tensor(tau, u, torch.from_numpy(xs[p]).to(dev), W.pairwise_secrets_for(u, ids), ids,
                                       weight=ws[p]) for p, u in enumerate(ids)])
    ref = O.lom_encrypt(xs[1].astype(np.float64), tau, ids[1], W.pairwise_secrets_for(ids[1], ids), ids, nonce,
                        weight=ws[1])
    assert np.array_equal(_u64(Y[1]), ref)
    out, sums = cr.aggregate_tensor(Y, sum(ws), want_sums=True)
    want = np.zeros(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for p in range(P):
            want += _qw(xs[p], ws[p])
    assert np.array_equal(_u64(sums), want)
    idx = np.random.default_rng(3).choice(n, 5000, replace=False)
    refo = O.reverse_quantize(O.apply_average([int(v) for v in want[idx]], sum(ws)))
    assert np.array_equal(out.cpu().numpy()[idx].view(np.uint64), refo.view(np.uint64))


def test_cfg4_jl_10m_8_parties_8_stripes(dev):
    """Config 4 on one GPU: the whole 10M-element vector and the 8 stripes each rank of an
    8-GPU element-range split owns (distributed.jl_shard, global ct_offset; reference
    _jls.py:473-505 encrypt, :646-699 aggregate)."""
    from fedbiomed_amd import distributed as Dd
    from fedbiomed_amd.secagg import SecaggCrypter

    n, P, tau, world = 10_000_000, 8, 1, 8
    ws = [W.party_weight(p) for p in range(P)]
    keys = [W.jl_user_key(p) for p in range(P)]
    sk0 = -sum(keys)
    es, cr_ = O.jl_slot(None, P)
    n_ct = (n + cr_ - 1) // cr_
    jc = SecaggCrypter()
    xs = [W.party_params(p, n) for p in range(P)]
    xd = [torch.from_numpy(x).to(dev) for x in xs]
    whole = torch.stack([jc.encrypt_tensor(P, tau, xd[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)])
    assert tuple(whole.shape) == (P, n_ct, 64)
    out_whole, sums = jc.aggregate_tensor(tau, whole, sk0, W.BIPRIME0, sum(ws), num_expected_params=n,
                                          want_sums=True)
    # the benchmark's path: every party's exponentiation and the decryption factor in ONE batched
    # launch (D.jl_exp_batch) -- bit-identical ciphertexts and aggregate
    with D.deferred_checks():
        pend = [jc.encrypt_tensor(P, tau, xd[p], keys[p], W.BIPRIME0, weight=ws[p], defer_exp=True) for p in range(P)]
        pf = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0, phased=True)
        with D.jl_exp_batch(dev):
            pf.exponentiate()
            cts = [q.finish() for q in pend]  # (valid after the batch's launch, at exit)
        factor = pf.finish()
    batched = torch.stack(cts)
    assert torch.equal(batched, whole)
    out_b = jc.aggregate_tensor(tau, batched, sk0, W.BIPRIME0, sum(ws), num_expected_params=n, decrypt_factor=factor)
    assert torch.equal(out_b, out_whole)
    del batched, cts, pend, pf, factor, out_b
    # the 8 stripes: ciphertexts and aggregates bit-identical to the whole vector's
    outs = []
    for r in range(world):
        lo, hi = Dd.jl_shard(n, world, r, cr_)
        k0, k1 = lo // cr_, (hi + cr_ - 1) // cr_
        cts = torch.stack([jc.encrypt_tensor(P, tau, xd[p][lo:hi], keys[p], W.BIPRIME0, weight=ws[p],
                                             ct_offset=k0) for p in range(P)])
        assert torch.equal(cts, whole[:, k0:k1]), r
        outs.append(jc.aggregate_tensor(tau, cts, sk0, W.BIPRIME0, sum(ws), num_expected_params=hi - lo,
                                        ct_offset=k0))
        del cts
    assert torch.equal(torch.cat(outs), out_whole)
    # sampled ciphertexts vs the oracle: every stripe's first and last ciphertext (so both sides of
    # each of the 7 cut points, the vector's first and its last, partial one), and random ones
    rng = np.random.default_rng(4)
    edges = set()
    for r in range(world):
        lo, hi = Dd.jl_shard(n, world, r, cr_)
        edges |= {lo // cr_, (hi + cr_ - 1) // cr_ - 1}
    assert len(edges) == 2 * world and {0, n_ct - 1} <= edges
    ks = sorted(edges | set(rng.choice(n_ct, 22, replace=False).tolist()))
    for p in range(P):
        got = D.limbs_to_ints(whole[p, ks].cpu().numpy())
        for k, g in zip(ks, got):
            qw = [int(v) for v in _qw(xs[p][k * cr_:(k + 1) * cr_], ws[p])]
            assert g == O.jl_encrypt_ints(qw, tau, keys[p], W.BIPRIME0, P, k0=k)[0], (p, k)
    # decoded integer sums exact over all 10M elements: sum_p q_p w_p
    sums = sums.cpu().numpy().view(np.uint64).reshape(n, 2)
    want = np.zeros(n, dtype=np.uint64)
    for p in range(P):
        want += _qw(xs[p], ws[p])
    assert (sums[:, 1] == 0).all() and np.array_equal(sums[:, 0], want)
    # every one of the 10M float64 outputs bit for bit against the oracle (so the batched and the 8 stripes'
    # outputs too: they equal this vector above)
    ref = _oracle_outputs(want, sum(ws))
    assert np.array_equal(out_whole.cpu().numpy().view(np.uint64), ref.view(np.uint64))


def _host_qw_sum(acc: np.ndarray, x: np.ndarray, w: int, threads: int = 8) -> None:
    """acc += O.quantize(x) * w (mod 2^64), on host threads over chunks (numpy releases the GIL):
    the oracle's quantise of a 100M-element vector in about a second instead of six."""
    from concurrent.futures import ThreadPoolExecutor

    step = -(-len(x) // threads)

    def part(a):
        with np.errstate(over="ignore"):
            acc[a:a + step] += O.quantize(x[a:a + step]) * np.uint64(w)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(part, range(0, len(x), step)))


def test_cfg5_lom_ass_100m_16_parties(dev):
    """Config 5 on one GPU: 16 parties' LOM protects of a 100M-element vector, the aggregate and
    the additive sharing of the sum.  Every expected value comes from the CPU oracle: the exact
    masked sum is sum_p quantize(x_p) * w_p computed on the host (_lom.py:105-175: the masks
    cancel), and every party's masked vector is checked bit for bit on windows at each cut point
    of an 8-GPU element-range split (distributed.lom_shard) and at both ends of the vector."""
    from fedbiomed_amd import distributed as Dd
    from fedbiomed_amd.secagg import AdditiveSecret, AdditiveShares, SecaggLomCrypter

    n, P, tau, world = 100_000_000, 16, 1, 8
    ids, ws = W.node_ids(P), [W.party_weight(p) for p in range(P)]
    nonce = O.lom_nonce(W.LOM_NONCE)
    cr = SecaggLomCrypter(W.LOM_NONCE)
    gen = torch.Generator(device=dev)
    Y = torch.empty((P, n), dtype=torch.int64, device=dev)
    want = np.zeros(n, dtype=np.uint64)  # the oracle's sum_p q_p w_p (mod 2^64)
    cuts = [Dd.lom_shard(n, world, r)[0] for r in range(1, world)]
    assert all(c % 8 == 0 for c in cuts)
    m = 512  # a window of m elements on each side of every cut point, and at both ends
    e0 = (n - m - 3) // 8 * 8  # (the window oracle starts on a ChaCha20 block: 8-aligned offsets)
    wins = [(0, m)] + [(c - m, 2 * m) for c in cuts] + [(e0, n - e0)]
    for p, u in enumerate(ids):
        gen.manual_seed(500 + p)
        x = torch.randn(n, generator=gen, device=dev, dtype=torch.float32) * 0.05
        x[:: 997] = 4.0 * (1 - 2 * (p & 1))  # clipped entries
        Y[p] = cr.encrypt_tensor(tau, u, x, W.pairwise_secrets_for(u, ids), ids, weight=ws[p])
        xh = x.cpu().numpy()
        _host_qw_sum(want, xh, ws[p])
        for off, k in wins:
            ref = _lom_window_oracle(u, ids, tau, _qw(xh[off:off + k], ws[p]), off, nonce)
            assert np.array_equal(_u64(Y[p, off:off + k]), ref), (p, off)
        del x, xh
    # masks cancel exactly over all 100M elements (u64 wrap == int64 wrap), against the host sum
    out, sums = cr.aggregate_tensor(Y, sum(ws), want_sums=True)
    assert np.array_equal(_u64(sums), want)
    # all 100M float64 outputs bit for bit against the oracle
    assert np.array_equal(out.cpu().numpy().view(np.uint64), _oracle_outputs(want, sum(ws)).view(np.uint64))
    idx = np.random.default_rng(5).choice(n, 64, replace=False)
    del Y, out
    # additive secret sharing of the 100M summed vector into 16 shares, and back: the exact column
    # sum (_additive_ss.py:252-267) is the oracle's sum again
    shares = AdditiveSecret.split_tensor(sums, P, unsigned=True)
    rec = AdditiveShares.reconstruct_tensor(shares)
    assert np.array_equal(_u64(rec[:, 0]), want) and bool((rec[:, 1] == 0).all())
    hi = shares[:-1, :, 1]
    assert bool(((hi == 0) | (hi == 1)).all())  # first P-1 shares in [0, 2^64]
    # a sampled column of shares summed on the host as Python ints (no modulus, as the reference)
    cols = shares[:, idx[:64]].cpu().numpy()
    for j, e in enumerate(idx[:64]):
        tot = sum(int(cols[q, j, 0]) % 2 ** 64 + (int(cols[q, j, 1]) << 64) for q in range(P))
        assert tot == int(want[e]), e
