"""FDH objects of any bits_size (round 4): the last object-API FDH shape the device path refused.

The reference's FDH(bits_size, M).H(t) (`_jls.py:742-762`) hashes int(t).to_bytes(bits_size // 2) || counter
and concatenates the digests until gcd(r, M) == 1.  Once r holds bits_size // 8 bytes its inner loop stops
breaking, so the counter byte overflows at 256: bits_size < 264 always raises OverflowError, and r has at
most ceil(bits_size / 256) - 1 digests.  The crypter uses FDH(2048, N^2) only (fbm_jl_fdh, fused in the
encrypt and the decryption factor).  Any other bits_size runs on `jl_fdh_msg_kernel` (fbm_jl_fdh_msg):
one lane per t, the message blocks hashed on the device.  Fixture: tests/golden/fdh_bits.json
(tools/gen_golden.py gen_fdh_bits, the reference's outcomes; bits_size 8 ... 4096 over a real biprime's
square, small odd, even, prime-power moduli and 1; t = 0, 1, random, the largest and the first too-large
message, -1).
"""

import pytest

from oracle import secagg_oracle as O
from tests.golden_util import I, load


@pytest.fixture(scope="module")
def fb():
    return load("fdh_bits.json")


def _cases(fb):
    for e in fb["fdh"]:
        for c in e["cases"]:
            yield e["bits"], I(e["m"]), I(c["t"]), c["h"]


def test_fdh_bits_oracle_vs_fixture(fb):
    """The oracle's restatement (any bits_size) against every reference outcome."""
    n = 0
    for bits, m, t, h in _cases(fb):
        if bits < 264 and "ok" not in h:  # the reference's 255-digest loop: its outcome is fixed
            assert h["error"] == "OverflowError"
            continue
        if "ok" in h:
            assert O.fdh_bits(t, m, bits) == I(h["ok"]), (bits, m, t)
            n += 1
        else:
            with pytest.raises(OverflowError) as ei:
                O.fdh_bits(t, m, bits)
            assert str(ei.value) == h["msg"]
    assert n > 300


@pytest.mark.gpu
def test_fdh_bits_device_vs_fixture(fb):
    """FDH(bits_size, M).H on the device (jl_fdh_msg_kernel through the object API) equals the reference
    for every case of the fixture: values, OverflowErrors (message too long, negative t, bits_size < 264,
    no coprime r), bit for bit -- r of up to 11 digests among them (M = 6 at 3072 bits).  r of 16 and more
    digests (bits_size > 4096): tests/test_fdh_wide.py."""
    from fedbiomed_amd.secagg._jls import FDH

    for bits, m, t, h in _cases(fb):
        f = FDH(bits, m)
        if "ok" in h:
            want = I(h["ok"])
            assert want.bit_length() <= 15 * 256, (bits, m, t)  # r of at most 15 digests
            assert f.H(t) == want, (bits, m, t)
        else:
            with pytest.raises(Exception) as ei:
                f.H(t)
            assert type(ei.value).__name__ == h["error"] and str(ei.value) == h["msg"], (bits, m, t, ei.value)


@pytest.mark.gpu
def test_fdh_bits_object_api_gpu(fb):
    """UserKey.encrypt / ServerKey.decrypt under PublicParam(123457, 1024, FDH(1024, N^2).H): the reference's
    ciphertexts and plaintexts (rounds 2 and 3 refused this hashing function with FB624)."""
    from fedbiomed_amd.secagg._jls import FDH, EncryptedNumber, PublicParam, ServerKey, UserKey

    c = fb["user_encrypt_fdh1024"]
    n = c["n"]
    pp = PublicParam(n, 1024, FDH(1024, n * n).H)
    cts = UserKey(pp, c["key"]).encrypt(c["pt"], c["tau"])
    assert cts == [I(v) for v in c["ct"]]
    assert ServerKey(pp, -c["key"]).decrypt([EncryptedNumber(pp, v) for v in cts], c["tau"]) == c["dec"]
