"""FDH objects whose r takes 16 or more digests (round 5; the last FDH shape round 4 refused with FB624).

For bits_size > 4096 the reference's inner loop (`_jls.py:742-762`) keeps breaking while r is shorter than
bits_size // 8 bytes, so r may take up to min(ceil(bits_size / 256) - 1, 255) digests -- the counter byte
overflows at 256.  On the device r that wide does not fit a lane's registers: `jl_fdh_msg_wide_kernel`
(fbm_jl.hip) writes each digest to the output row as it is made and decides gcd(r, M) == 1 on r R mod m,
updated per digest with two Montgomery products (m the modulus's odd part); rows are
fbm_jl_fdh_msg_row_words(bits_size) words (ABI 4).  Fixture: tests/golden/fdh_wide.json (tools/gen_golden.py
gen_fdh_wide, the reference's outcomes over primorial moduli, where most candidates fail, up to 22 digests and
one OverflowError after 16)."""

import pytest

from oracle import secagg_oracle as O
from tests.golden_util import I, load


@pytest.fixture(scope="module")
def fw():
    return load("fdh_wide.json")


def _cases(fw):
    for e in fw:
        for c in e["cases"]:
            yield e["bits"], I(e["m"]), I(c["t"]), c["h"]


def test_fdh_wide_fixture_reaches_16_digests(fw):
    wide = [I(h["ok"]) for _, _, _, h in _cases(fw) if "ok" in h and I(h["ok"]).bit_length() > 15 * 256]
    assert len(wide) >= 3
    assert any("error" in h for _, _, _, h in _cases(fw))


def test_fdh_wide_oracle_vs_fixture(fw):
    for bits, m, t, h in _cases(fw):
        if "ok" in h:
            assert O.fdh_bits(t, m, bits) == I(h["ok"]), (bits, t)
        else:
            with pytest.raises(OverflowError):
                O.fdh_bits(t, m, bits)


def test_row_words_abi():
    """fbm_jl_fdh_msg_row_words: 128 words up to 15 digests, 8 per digest above, 255 digests at most
    (host-side, no device call)."""
    from fedbiomed_amd import _native

    lib = _native.load_host_only() if hasattr(_native, "load_host_only") else None
    if lib is None:
        import ctypes

        lib = ctypes.CDLL(_native.lib_path())
        lib.fbm_jl_fdh_msg_row_words.restype = ctypes.c_int
        lib.fbm_jl_fdh_msg_row_words.argtypes = [ctypes.c_int]
    assert lib.fbm_jl_fdh_msg_row_words(2048) == 128
    assert lib.fbm_jl_fdh_msg_row_words(4096) == 128
    assert lib.fbm_jl_fdh_msg_row_words(4104) == 8 * 16
    assert lib.fbm_jl_fdh_msg_row_words(8192) == 8 * 31
    assert lib.fbm_jl_fdh_msg_row_words(70000) == 8 * 255


@pytest.mark.gpu
def test_fdh_wide_device_vs_fixture(fw):
    from fedbiomed_amd.secagg._jls import FDH

    for bits, m, t, h in _cases(fw):
        f = FDH(bits, m)
        if "ok" in h:
            assert f.H(t) == I(h["ok"]), (bits, m, t)
        else:
            with pytest.raises(Exception) as ei:
                f.H(t)
            assert type(ei.value).__name__ == h["error"] and str(ei.value) == h["msg"], (bits, t, ei.value)


@pytest.mark.gpu
def test_fdh_wide_batch_equals_single(fw):
    """One launch over every t of a modulus (_hash_range's path) equals the per-t calls."""
    from fedbiomed_amd import _device as D

    e = next(x for x in fw if x["bits"] == 8192 and I(x["m"]) % 2 == 0 and I(x["m"]) != 2**20)
    ts = [I(c["t"]) for c in e["cases"]]
    h = D.jl_fdh_msg(ts, e["bits"], I(e["m"]))
    got = D.limbs_to_ints_w(h, h.shape[1])
    assert got == [I(c["h"]["ok"]) for c in e["cases"]]
