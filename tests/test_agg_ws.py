"""The wave-split aggregate kernels of round 5 at the edges of their tiles (`lom_aggregate_ws_kernel` for 8 and 16
parties: 128-element tiles, the last one bounds-checked; `ass_reconstruct_ws_kernel` for 16 shares: 64-element
tiles), and the shapes that keep the round-4 kernels (an odd length, a row start that is not 16-byte aligned,
other party counts): every output -- the float64 average, the u64 sums -- bit-identical to the oracle's
LOM.aggregate + _apply_average + reverse_quantize (`secagg/_lom.py:177-192`, `_secagg_crypter.py:233-249`,
`utils/_secagg_utils.py:152-187`) and to the exact int128 sums (`_additive_ss.py:252-267`)."""

import numpy as np
import pytest

from oracle import secagg_oracle as O


def _rows(rng, P, n):
    # masked-looking u64 rows whose column sums cancel to small quantised values (as a real LOM round's)
    y = rng.integers(0, 2**63, size=(P, n), dtype=np.uint64) * np.uint64(2)
    target = rng.integers(0, 8191 * 1000, size=n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        y[P - 1] = target - np.sum(y[:P - 1], axis=0, dtype=np.uint64)
    return y


@pytest.mark.gpu
@pytest.mark.parametrize("P", [8, 16, 5])
@pytest.mark.parametrize("n", [1, 2, 127, 128, 130, 1001, 4098, 100_066])
def test_lom_aggregate_tiles_vs_oracle(P, n):
    import torch

    from fedbiomed_amd import _device as D

    rng = np.random.default_rng(1000 * P + n)
    y = _rows(rng, P, n)
    tw = 1000 * P + 17
    want_sums = O.lom_aggregate(y)
    want = O.lom_crypter_aggregate(y, tw)
    Y = torch.from_numpy(y.view(np.int64)).to(D.device())
    out, sums = D.lom_aggregate(Y, tw, want_out=True, want_sums=True)
    assert np.array_equal(sums.cpu().numpy().view(np.uint64), want_sums)
    assert np.array_equal(out.cpu().numpy().view(np.uint64), np.asarray(want, dtype=np.float64).view(np.uint64))
    only, _ = D.lom_aggregate(Y, tw, want_out=True, want_sums=False)
    assert torch.equal(only, out)
    _, only_sums = D.lom_aggregate(Y, tw, want_out=False, want_sums=True)
    assert torch.equal(only_sums, sums)


@pytest.mark.gpu
@pytest.mark.parametrize("P", [8, 16])
def test_lom_aggregate_unaligned_rows(P):
    """A [P, n] view whose rows start off a 16-byte boundary takes the round-4 kernel: same results."""
    import torch

    from fedbiomed_amd import _device as D

    rng = np.random.default_rng(77 + P)
    n = 4097
    y = _rows(rng, P, n + 1)
    big = torch.from_numpy(np.ascontiguousarray(y.view(np.int64).reshape(-1))).to(D.device())
    Y = big[1:1 + P * n].view(P, n)  # 8-byte offset, odd length
    ref = Y.cpu().numpy().view(np.uint64)
    out, sums = D.lom_aggregate(Y, 999, want_out=True, want_sums=True)
    assert np.array_equal(sums.cpu().numpy().view(np.uint64), O.lom_aggregate(ref))
    assert np.array_equal(out.cpu().numpy(), np.asarray(O.lom_crypter_aggregate(ref, 999), dtype=np.float64))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 65_537])
def test_ass_reconstruct_16_shares_tiles(n):
    import torch

    from fedbiomed_amd import _device as D

    rng = np.random.default_rng(n)
    secret = rng.integers(-(2**63), 2**63 - 1, size=n, dtype=np.int64)
    s = torch.from_numpy(secret).to(D.device())
    shares = D.ass_split(s, 16)
    rec = D.ass_reconstruct(shares)
    lo = rec[:, 0].cpu().numpy()
    hi = rec[:, 1].cpu().numpy()
    assert np.array_equal(lo, secret)
    assert np.array_equal(hi, np.where(secret < 0, -1, 0))
    # the exact int128 column sum of the shares themselves (the oracle's reconstruct)
    sh = shares.cpu().numpy()
    k = np.random.default_rng(1).choice(n, size=min(n, 50), replace=False)
    for i in k:
        v = sum((int(sh[p, i, 1]) << 64) + (int(sh[p, i, 0]) & (2**64 - 1)) for p in range(16))
        v = ((v + 2**127) % 2**128) - 2**127
        assert v == int(secret[i])
