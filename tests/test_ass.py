"""Additive secret sharing of vectors (reference secagg/_additive_ss.py).

Contract (the reference draws from MT19937, which is not part of it): split shares sum
exactly to the secret and the first n-1 lie in [0, 2**bit_length] (bit_length = the
secret's bit length unless given); reconstruct is an exact column sum -- checked against
the reference's own shares in tests/golden/ass.json.
"""

import numpy as np
import pytest
import torch

from fedbiomed_amd import _device as D
from tests.golden_util import I


# ---- CPU: host-side int128 conversions and validation --------------------------------------
def test_int128_roundtrip():
    vals = [0, 1, -1, 2**63, -(2**63), 2**64 + 5, -(2**70) + 3, 2**127 - 1, -(2**127)]
    assert D.int128_to_ints(D.ints_to_int128(vals)) == vals
    with pytest.raises(ValueError):
        D.ints_to_int128([2**127])


def test_validation_matches_reference():
    from fedbiomed_amd.exceptions import FedbiomedTypeError, FedbiomedValueError
    from fedbiomed_amd.secagg import AdditiveSecret, AdditiveShare, AdditiveShares

    with pytest.raises(FedbiomedValueError):
        AdditiveSecret("x")
    with pytest.raises(FedbiomedValueError):
        AdditiveSecret([1, 2.0])
    with pytest.raises(FedbiomedValueError):
        AdditiveSecret(5).split(0)
    with pytest.raises(FedbiomedValueError):  # bit_length < int(log2(secret))
        AdditiveSecret(2**40).split(3, bit_length=8)
    with pytest.raises(FedbiomedTypeError):
        AdditiveShare("a")
    with pytest.raises(FedbiomedTypeError):
        AdditiveShares([1, 2])
    with pytest.raises(FedbiomedTypeError):
        AdditiveShare(1) + AdditiveShare([1])
    with pytest.raises(FedbiomedTypeError):
        AdditiveShares([AdditiveShare(1)]) + AdditiveShares([AdditiveShare(1), AdditiveShare(2)])


# ---- GPU -------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return D.device()


@pytest.mark.gpu
def test_reconstruct_reference_shares(golden, dev):
    """Reconstruct the reference's own shares (int and list secrets) bit-exactly."""
    from fedbiomed_amd.exceptions import FedbiomedValueError
    from fedbiomed_amd.secagg import AdditiveShare, AdditiveShares

    for case in golden["ass"]["cases"]:
        sh = case["shares"]
        if isinstance(sh[0], list):
            shares = AdditiveShares([AdditiveShare([I(x) for x in s]) for s in sh])
            want = [I(x) for x in case["reconstruct"]]
        else:
            shares = AdditiveShares([AdditiveShare(I(s)) for s in sh])
            want = I(case["reconstruct"])
        if max(abs(I(x)) for s in sh for x in (s if isinstance(s, list) else [s])) >= 2**126:
            with pytest.raises(FedbiomedValueError):  # 2040-bit key shares: reference-side only
                shares.reconstruct()
            continue
        assert shares.reconstruct() == want
        assert sum(shares).value == want  # __radd__/__add__ path (a single AdditiveShare)


@pytest.mark.gpu
@pytest.mark.parametrize("unsigned", [False, True])
def test_split_invariants_large(dev, unsigned):
    rng = np.random.default_rng(11)
    n, P = 1_000_003, 16
    if unsigned:
        x = rng.integers(0, 2**64, size=n, dtype=np.uint64)
        x[:4] = [0, 1, 2**64 - 1, 2**63]
        sec = torch.from_numpy(x.view(np.int64)).to(dev)
    else:
        x = rng.integers(-(2**63), 2**63, size=n, dtype=np.int64)
        x[:5] = [0, -1, 1, -(2**63), 2**63 - 1]
        x[5:1000] = rng.integers(-1000, 1000, size=995)
        sec = torch.from_numpy(x).to(dev)
    shares = D.ass_split(sec, P, unsigned=unsigned)
    rec = D.ass_reconstruct(shares).cpu().numpy()
    # exact sum == secret (as int128)
    want = D.ints_to_int128([int(v) for v in x.tolist()])
    assert np.array_equal(rec, want)
    # ranges: first P-1 shares in [0, 2^b], b = bit length of |v|
    s = shares.cpu().numpy()[:-1]  # [P-1, n, 2]
    mag = np.array([abs(int(v)) for v in x[:20000].tolist()], dtype=object)
    bl = np.array([int(m).bit_length() for m in mag])
    lo, hi = s[:, :20000, 0].view(np.uint64), s[:, :20000, 1]
    assert (hi >= 0).all() and (hi <= 1).all()
    full = [[(int(h) << 64) | int(l) for l, h in zip(lo[p].tolist(), hi[p].tolist())] for p in range(P - 1)]
    for p in range(P - 1):
        assert all(0 <= full[p][i] <= (1 << int(bl[i])) for i in range(20000))
    # not degenerate: shares of 64-bit-wide secrets spread over their range
    wide = bl == 64
    if wide.any():
        col = np.array([full[0][i] for i in np.nonzero(wide)[0]], dtype=object)
        assert len(set(col.tolist())) == len(col)


@pytest.mark.gpu
def test_split_bit_length_and_offsets(dev):
    from fedbiomed_amd.secagg import AdditiveSecret

    x = torch.arange(1, 5001, dtype=torch.int64, device=dev)
    seed, nonce = bytes(range(32)), b"abcdefgh"
    whole = D.ass_split(x, 5, bit_length=20, seed=seed, nonce=nonce)
    assert int(whole[:-1, :, 1].abs().max()) == 0 and int(whole[:-1, :, 0].max()) <= 2**20
    parts = [D.ass_split(x[a:b], 5, bit_length=20, seed=seed, nonce=nonce, elem_offset=a)
             for a, b in [(0, 1000), (1000, 4321), (4321, 5000)]]
    assert torch.equal(torch.cat(parts, dim=1), whole)
    # list API round trip, scalar and list secrets
    sh = AdditiveSecret([5, 2**63 + 7, 0, 123]).split(4)
    assert len(sh) == 4 and sh.reconstruct() == [5, 2**63 + 7, 0, 123]
    sh = AdditiveSecret(12345678901234567890).split(3)
    assert isinstance(sh[0].value, int) and sh.reconstruct() == 12345678901234567890
    assert AdditiveSecret([-7, 9]).split(2, bit_length=None).reconstruct() == [-7, 9]
