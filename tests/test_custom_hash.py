"""The JoyeLibert object API under a PublicParam whose hashing function is not FDH(2048, N^2).H
(reference _jls.py:451-467: BaseKey._populate_tau calls the PublicParam's callable per t, and
UserKey.encrypt / ServerKey.decrypt raise its values to the key with gmpy2.powmod, :473-562).  The
mirror calls the callable on the host as the reference does and runs the exponentiations on the device
(fbm_jl_powmod, fbm_jl_decrypt_with).  Pinned by tests/golden/custom_hash.json -- the reference's own
outputs for the callables of tests/golden_util.custom_hashes() and an FDH against N, over an odd
biprime, a small odd and an even modulus, rounds inside and outside FDH's range (a callable takes any
t), positive and negative keys (tools/gen_golden.py gen_custom_hash)."""

import pytest

from fedbiomed_amd.secagg._jls import FDH, EncryptedNumber, JoyeLibert, PublicParam, ServerKey, UserKey
from oracle import secagg_oracle as O
from tests.golden_util import I, custom_hashes


def _hash_fn(case, api: bool):
    n = I(case["n"])
    if case["hash"] == "fdh_n":  # FDH(2048, N).H: gcd against N, not N^2
        return FDH(2048, n).H if api else (lambda t: O.fdh(t, n))
    return custom_hashes()[case["hash"]]


def _cases(golden):
    return golden["custom_hash"]["cases"]


# ------------------------------------------------------------------ CPU: the oracle against the reference
def test_oracle_matches_reference_fixture(golden):
    """The oracle's UserKey.encrypt / ServerKey.decrypt with the PublicParam's callable equal the
    reference's outputs (and its OverflowError where the callable raises)."""
    for case in _cases(golden):
        n, tau, (k1, k2) = I(case["n"]), case["tau"], case["keys"]
        hf = _hash_fn(case, api=False)
        pts, pts2 = [I(v) for v in case["pts"]], [I(v) for v in case["pts2"]]
        for pt, k, enc in ((pts, k1, case["enc1"]), (pts2, k2, case["enc2"])):
            if "ok" in enc:
                assert O.jl_user_encrypt(pt, tau, k, n, hashing_function=hf) == [I(c) for c in enc["ok"]], case["hash"]
            else:
                with pytest.raises(OverflowError):
                    O.jl_user_encrypt(pt, tau, k, n, hashing_function=hf)
        if "ok" in case.get("dec", {}):
            sums = [I(a) * I(b) % (n * n) for a, b in zip(case["enc1"]["ok"], case["enc2"]["ok"])]
            got = O.jl_server_decrypt(sums, tau, case["sk0"], n, hashing_function=hf)
            assert got == [I(v) for v in case["dec"]["ok"]]
            assert got == [(a + b) % n for a, b in zip(pts, pts2)]


def test_fdh_of_another_bits_size_checks_its_message_on_the_host():
    """FDH of bits_size other than 2048 runs on the device since round 4 (tests/test_fdh_bits.py); its
    to_bytes errors come first, on the host, as the reference's int(t).to_bytes(bits_size // 2) raises them
    (messages pinned in tests/golden/fdh_bits.json)."""
    f = FDH(1024, 123457 ** 2)
    with pytest.raises(OverflowError, match="can't convert negative int to unsigned"):
        f.H(-1)
    with pytest.raises(OverflowError, match="int too big to convert"):
        f.H(1 << (8 * 512))
    with pytest.raises(ValueError, match="length argument must be non-negative"):
        FDH(-2, 7).H(1)


# ------------------------------------------------------------------ GPU: the device path against the reference
@pytest.mark.gpu
def test_user_encrypt_server_decrypt_match_reference(golden):
    for case in _cases(golden):
        n, tau, (k1, k2) = I(case["n"]), case["tau"], case["keys"]
        pp = PublicParam(n, 1024, _hash_fn(case, api=True))
        pts, pts2 = [I(v) for v in case["pts"]], [I(v) for v in case["pts2"]]
        for pt, k, enc in ((pts, k1, case["enc1"]), (pts2, k2, case["enc2"])):
            if "ok" in enc:
                assert UserKey(pp, k).encrypt(pt, tau) == [I(c) for c in enc["ok"]], (case["hash"], n, tau)
            else:
                with pytest.raises(OverflowError):
                    UserKey(pp, k).encrypt(pt, tau)
        if "dec" not in case:
            continue
        ens = [EncryptedNumber(pp, I(a)) + EncryptedNumber(pp, I(b)) for a, b in zip(case["enc1"]["ok"], case["enc2"]["ok"])]
        if "ok" in case["dec"]:
            assert ServerKey(pp, case["sk0"]).decrypt(ens, tau) == [I(v) for v in case["dec"]["ok"]]
        else:  # a base with no inverse under a negative key (parity unpinned: the error type, see the docstring)
            with pytest.raises((ZeroDivisionError, ValueError)):
                ServerKey(pp, case["sk0"]).decrypt(ens, tau)


@pytest.mark.gpu
def test_protect_aggregate_match_reference(golden):
    for case in _cases(golden):
        if "protect" not in case:
            continue
        n, tau, (k1, k2), g = I(case["n"]), case["tau"], case["keys"], case["protect"]
        pp = PublicParam(n, 1024, _hash_fn(case, api=True))
        jl = JoyeLibert()
        y1 = jl.protect(pp, UserKey(pp, k1), tau, g["x1"], 2)
        y2 = jl.protect(pp, UserKey(pp, k2), tau, g["x2"], 2)
        assert y1 == [I(c) for c in g["y1"]] and y2 == [I(c) for c in g["y2"]], (case["hash"], n, tau)
        ys = [[EncryptedNumber(pp, c) for c in y] for y in (y1, y2)]
        if "ok" in g["agg"]:
            assert jl.aggregate(ServerKey(pp, case["sk0"]), tau, ys, 9) == g["agg"]["ok"]
            if n.bit_length() > 1000:  # small moduli wrap the packed plaintext (as in the reference)
                assert g["agg"]["ok"] == [a + b for a, b in zip(g["x1"], g["x2"])]
        else:
            with pytest.raises((ZeroDivisionError, ValueError)):
                jl.aggregate(ServerKey(pp, case["sk0"]), tau, ys, 9)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["auto", "generic"])
def test_custom_hash_sweep_against_oracle(engine):
    """A longer vector (300 plaintexts) of the 2048-bit SHA-based callable over the benchmark biprime,
    positive and negative keys, on the Montgomery engines and on the generic one."""
    import random

    from fedbiomed_amd import _device as D, workload as W

    rng = random.Random(7)
    n = W.BIPRIME0
    hf = custom_hashes()["sha"]
    pp = PublicParam(n, 1024, hf)
    pts = [rng.randrange(n) for _ in range(300)]
    with D.jl_engine(engine):
        for key in (W.jl_user_key(1), -W.jl_user_key(2)):
            assert UserKey(pp, key).encrypt(pts, 11) == O.jl_user_encrypt(pts, 11, key, n, hashing_function=hf)
        cts = UserKey(pp, W.jl_user_key(3)).encrypt(pts, 11)
        got = ServerKey(pp, -W.jl_user_key(3)).decrypt([EncryptedNumber(pp, c) for c in cts], 11)
    assert got == pts
