"""Additive secret sharing of vectors (reference secagg/_additive_ss.py).

Contract: split shares sum exactly to the secret and the first n-1 lie in [0, 2**bit_length]
(bit_length = the secret's bit length unless given); reconstruct is an exact column sum -- checked
against the reference's own shares in tests/golden/ass.json.  An int secret's shares are the
reference's own MT19937 draws (seeded as the fixture was made); a vector's come from ChaCha20.
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
def test_int_split_is_the_reference_stream(golden, dev):
    """With reference_rng=True an int secret (the key setup's use) draws its shares from Python's MT19937
    call for call: seeded as tools/gen_golden.py seeded the reference, the shares are the reference's own
    (the 64- and 2040-bit cases of tests/golden/ass.json), and `random` is left where the reference leaves
    it; a vector secret does too (the fixture's list case)."""
    import random

    from fedbiomed_amd.secagg import AdditiveSecret

    cases = [c for c in golden["ass"]["cases"] if not isinstance(c["secret"], list)]
    assert len(cases) == 2
    for case in cases:
        secret, n = I(case["secret"]), len(case["shares"])
        random.seed(99)
        assert AdditiveSecret(secret).split(n, reference_rng=True).to_list() == [I(s) for s in case["shares"]]
        after = random.getstate()
        random.seed(99)
        for _ in range(n - 1):
            random.randint(0, 2**secret.bit_length())
        assert random.getstate() == after
    # a vector secret with reference_rng (an extension): the reference's list case, share for share
    (case,) = [c for c in golden["ass"]["cases"] if isinstance(c["secret"], list)]
    random.seed(99)
    got = AdditiveSecret([I(v) for v in case["secret"]]).split(len(case["shares"]), reference_rng=True)
    assert got.to_list() == [[I(x) for x in s] for s in case["shares"]]
    random.seed(3)  # and wide, negative and bit_length-given vectors keep the contract
    vals = [2**200 + 1, -(2**90), 0, 7]
    sh = AdditiveSecret(vals).split(5, reference_rng=True)
    assert sh.reconstruct() == vals and all(0 <= v <= 2**abs(x).bit_length() for s in sh.to_list()[:-1]
                                            for v, x in zip(s, vals))
    assert AdditiveSecret([5, 6]).split(3, bit_length=70, reference_rng=True).reconstruct() == [5, 6]
    random.seed(7)
    assert AdditiveSecret(-12345).split(1, reference_rng=True).to_list() == [-12345]
    assert AdditiveSecret(2**70).split(3, bit_length=100, reference_rng=True).reconstruct() == 2**70


@pytest.mark.gpu
def test_int_split_default_is_not_the_mt19937_stream(golden, dev):
    """by default an int secret -- a node's 2040-bit JL key at setup -- draws its shares
    from the device's OS-keyed ChaCha20, never from `random`: the global stream is left untouched, two
    splits of the same secret under the same seed differ, and the contract holds (exact sum, the first
    n - 1 shares in [0, 2**bit_length])."""
    import random

    from fedbiomed_amd.secagg import AdditiveSecret

    for case in [c for c in golden["ass"]["cases"] if not isinstance(c["secret"], list)]:
        secret, n = I(case["secret"]), len(case["shares"])
        random.seed(99)
        before = random.getstate()
        a = AdditiveSecret(secret).split(n).to_list()
        assert random.getstate() == before  # no draw from the reference's MT19937
        assert a != [I(s) for s in case["shares"]]
        random.seed(99)
        b = AdditiveSecret(secret).split(n).to_list()
        assert a != b
        for sh in (a, b):
            assert sum(sh) == secret and all(0 <= v <= 2**secret.bit_length() for v in sh[:-1])
    assert AdditiveSecret(-12345).split(1).to_list() == [-12345]
    assert AdditiveSecret(2**70).split(3, bit_length=100).reconstruct() == 2**70


def test_reference_stream_draws_match_fixture(golden):
    """CPU: the draws alone (D.reference_share_draws, the C MT19937 replay) against the reference's own
    shares from tests/golden/ass_stream.json, seeded as the reference was, and the stream's next 64 bits."""
    import random

    for case in golden["ass_stream"]["cases"]:
        secret = case["secret"]
        if not isinstance(secret, list):
            continue  # (an int secret's draws are `random.randint` itself)
        vals = [I(v) for v in secret]
        bls = [v.bit_length() if case["bit_length"] is None else case["bit_length"] for v in vals]
        random.seed(case["seed"])
        rows = D.reference_share_draws(bls, case["n"] - 1)
        assert rows == [[I(x) for x in s] for s in case["shares"][:-1]], case["seed"]
        assert random.getrandbits(64) == I(case["next_getrandbits64"]), case["seed"]


@pytest.mark.gpu
def test_split_reference_stream_fixture(golden, dev):
    """The reference's seeded splits (tests/golden/ass_stream.json: vectors of mixed widths and signs, a given
    bit_length, an int secret with bit_length 300, a value past 126 bits) share for share, last share
    included, and `random` left where the reference left it."""
    import random

    from fedbiomed_amd.secagg import AdditiveSecret

    for case in golden["ass_stream"]["cases"]:
        secret = case["secret"]
        secret = [I(v) for v in secret] if isinstance(secret, list) else I(secret)
        random.seed(case["seed"])
        sh = AdditiveSecret(secret).split(case["n"], case["bit_length"], reference_rng=True)
        want = [[I(x) for x in s] if isinstance(s, list) else I(s) for s in case["shares"]]
        assert sh.to_list() == want, case["seed"]
        assert random.getrandbits(64) == I(case["next_getrandbits64"]), case["seed"]


@pytest.mark.gpu
def test_reconstruct_reference_shares(golden, dev):
    """Reconstruct the reference's own shares (int and list secrets) bit-exactly."""
    from fedbiomed_amd.secagg import AdditiveShare, AdditiveShares

    for case in golden["ass"]["cases"]:
        sh = case["shares"]
        if isinstance(sh[0], list):
            shares = AdditiveShares([AdditiveShare([I(x) for x in s]) for s in sh])
            want = [I(x) for x in case["reconstruct"]]
        else:
            shares = AdditiveShares([AdditiveShare(I(s)) for s in sh])
            want = I(case["reconstruct"])
        assert shares.reconstruct() == want  # incl. the 2040-bit key shares (wide limb path)
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


@pytest.mark.gpu
def test_split_wide_key_setup(dev):
    """The JL key setup's use (node/secagg/_secagg_setups.py:248-268): a 2040-bit user key
    split into one share per party, the shares summed back -- and wide vectors, negative
    values, explicit bit lengths, shard offsets."""
    import random

    from fedbiomed_amd.secagg import AdditiveSecret, AdditiveShare, AdditiveShares

    rnd = random.Random(5)
    for P in (1, 2, 3, 8, 17):
        sk = rnd.getrandbits(2040)
        shares = AdditiveSecret(sk).split(P).to_list()
        assert len(shares) == P and sum(shares) == sk
        b = sk.bit_length()
        assert all(0 <= v <= 2**b for v in shares[:-1])
        # the setup's own sequence: last share kept, the others summed as AdditiveShares
        mine = AdditiveShare(shares.pop(-1))
        if not shares:  # one party: sum([]) == 0 and share + 0 raises, as in the reference
            continue
        assert (mine + sum(AdditiveShares([AdditiveShare(v) for v in shares]))).value == sk
    # server key: sum of negative 2040-bit shares (researcher/secagg/_secagg_context.py:380)
    neg = [-rnd.getrandbits(2040) for _ in range(5)]
    assert AdditiveShares([AdditiveShare(v) for v in neg]).reconstruct() == sum(neg)
    # list secrets beyond 64 bits, mixed signs, bit_length given
    vals = [0, 1, -1, 2**64, -(2**64) - 5, 2**200 + 3, -(2**130)]
    sh = AdditiveSecret(vals).split(4)
    assert sh.reconstruct() == vals
    sh = AdditiveSecret([2**70, 5]).split(3, bit_length=300)
    assert sh.reconstruct() == [2**70, 5]
    assert all(0 <= v <= 2**300 for s in sh.to_list()[:-1] for v in s)
    # device tensors: shards with element offsets reproduce the unsharded draw
    vals = [rnd.getrandbits(500) - 2**499 for _ in range(3000)]
    sec = torch.from_numpy(D.ints_to_limbs_tc(vals, 17)).to(dev)
    seed, nonce = bytes(range(32)), b"12345678"
    whole = D.ass_split_wide(sec, 6, 18, seed=seed, nonce=nonce)
    parts = [D.ass_split_wide(sec[:, a:b], 6, 18, seed=seed, nonce=nonce, elem_offset=a)
             for a, b in [(0, 1000), (1000, 2999), (2999, 3000)]]
    assert torch.equal(torch.cat(parts, dim=2), whole)
    assert D.limbs_tc_to_ints(D.ass_reconstruct_wide(whole).cpu().numpy()) == vals
    first = D.limbs_tc_to_ints(whole[0].cpu().numpy())
    assert all(0 <= v <= 2**abs(x).bit_length() for v, x in zip(first, vals))
    assert len(set(first)) > 2990  # draws are not degenerate


def test_wide_limb_roundtrip_and_draw_map():
    """Host checks of the wide path's conversions and of the share-draw map the kernel
    uses: r = (x >> 64) + [x mod 2^64 + (x >> b) >= 2^64] == floor(x (2^b + 1) / 2^(b+64))."""
    import random

    vals = [0, 1, -1, 2**64, -(2**64) - 5, 2**200 + 3, -(2**130), 2**255 - 1, -(2**255)]
    assert D.limbs_tc_to_ints(D.ints_to_limbs_tc(vals, 8)) == vals
    rnd = random.Random(3)
    for b in (0, 1, 31, 32, 33, 63, 64, 65, 100, 2040):
        for _ in range(200):
            x = rnd.getrandbits(b + 64)
            carry = int((x & (2**64 - 1)) + (x >> b) >= 2**64)
            r = (x >> 64) + carry
            assert r == (x * (2**b + 1)) >> (b + 64) and 0 <= r <= 2**b


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["int", "list"])
def test_share_exchange_flows(dev, kind):
    """reference tests/test_additive_ss.py:90-180: share addition, and the key setup's exchange
    (every user splits its key in 3, keeps one share, sends the others; the sums of what each
    user holds reconstruct the sum of the keys)."""
    import random

    from fedbiomed_amd.exceptions import FedbiomedTypeError
    from fedbiomed_amd.secagg import AdditiveSecret, AdditiveShares

    if kind == "int":
        assert (AdditiveSecret(10).split(2) + AdditiveSecret(15).split(2)).reconstruct() == 25
        with pytest.raises(FedbiomedTypeError):
            AdditiveSecret(10).split(2) + AdditiveSecret([1, 2, 3]).split(2)
    else:
        assert (AdditiveSecret([1, 2, 3]).split(3) + AdditiveSecret([4, 5, 6]).split(3)).reconstruct() == [5, 7, 9]
    rnd = random.Random(11)
    keys = [rnd.randint(0, 2**2048) if kind == "int" else [rnd.randint(0, 2**50) for _ in range(10)]
            for _ in range(3)]
    shares = [AdditiveSecret(k).split(3) for k in keys]
    held = [shares[u][u] + shares[(u + 1) % 3][u] + shares[(u + 2) % 3][u] for u in range(3)]
    got = AdditiveShares(held).reconstruct()
    assert got == (sum(keys) if kind == "int" else [sum(c) for c in zip(*keys)])
