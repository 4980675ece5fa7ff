"""N = 1, the last biprime the reference computes with that the device path refused (round 4).

The reference reduces everything modulo N^2 = 1: every ciphertext and every product of ciphertexts
is 0, FDH(2048, 1).H is the first digest (gcd(r, 1) = 1), and ServerKey.decrypt's
invert(delta^2, N^2) (`_jls.py:36-58,556`) raises ZeroDivisionError: its result modulo 1 is 0, which
the reference's own `invert` refuses -- an empty list included.  Here N = 1 takes the generic engine
(csrc/fbm_gen.hip: Barrett products modulo M = 1), and every decryption entry point returns
FBM_E_INVERSE.  Fixture: tests/golden/n_one.json (tools/gen_golden.py gen_n_one, the reference's
outcomes).  A negative key inverts H(t) modulo 1 before the power: gmpy2 is absent, so those cases
follow Python's pow(h, -1, 1) = 0 (the shim's) -- parity unpinned for them, as the fixture notes.
"""

import logging

import numpy as np
import pytest

from oracle import secagg_oracle as O
from tests.golden_util import F, I, load


@pytest.fixture(scope="module")
def n1():
    return load("n_one.json")


def _run(outcome, fn):
    if "error" in outcome:
        with pytest.raises(Exception) as ei:
            fn()
        assert type(ei.value).__name__ == outcome["error"]
        assert str(ei.value) == outcome["msg"]
        return None
    return fn()


# ------------------------------------------------------------------ CPU
def test_n_one_oracle_vs_fixture(n1):
    """The oracle restates the reference at N = 1: zero ciphertexts, the decryption's ZeroDivisionError."""
    for c in n1["crypter"]:
        got = O.jl_encrypt([F(v) for v in c["x"]], 1, I(c["key"]), 1, 2, weight=c["weight"])
        assert got == [I(v) for v in c["enc"]["ok"]]
        cts = [got, got]
        _run(c["agg"], lambda: O.jl_crypter_aggregate(cts, 1, -I(c["key"]), 1, 4, len(c["x"])))
    o = n1["object"]
    assert O.jl_user_encrypt([1, 5, 0], 1, 3, 1) == [I(v) for v in o["user_encrypt"]["ok"]]
    assert O.jl_user_encrypt([4], 1, 0, 1) == [I(v) for v in o["user_encrypt_zero_key"]["ok"]]
    assert O.fdh(5, 1) == I(o["fdh"]["ok"])
    _run(o["decrypt"], lambda: O.jl_server_decrypt([0], 1, -3, 1))
    _run(o["decrypt_empty"], lambda: O.jl_server_decrypt([], 1, -3, 1))


def test_n_one_generic_engine_host():
    """The generic engine's per-ciphertext arithmetic at M = 1 (host test hooks): every power -- a zero
    key's h^0 included -- every encrypt and every product is 0."""
    from tests.test_even_moduli import _Host

    h = _Host()
    for key in (0, 1, 12345, -77, 2**2040 - 5):
        for pt in (None, 0, 5, 2**1000 + 1):
            assert h.exp(0x1234567890ABCDEF << 200, key, 1, pt=pt) == 0, (key, pt)
    assert h.combine([0, 0, 0], 1) == 0
    assert h.combine([0], 1, factor=0, decrypt=True) == 0


def test_n_one_in_domain():
    from fedbiomed_amd import _device as D
    from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError

    assert int(D._biprime_limbs(1)[0]) == 1
    for n in (0, -4, 2**1024):
        with pytest.raises(FedbiomedSecaggCrypterError, match="FB624"):
            D._biprime_limbs(n)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_n_one_crypter_gpu(n1, caplog):
    """SecaggCrypter.encrypt at N = 1 (keys 0, positive, 2040-bit and negative, weighted or not):
    the reference's zero ciphertexts; aggregate: its ZeroDivisionError."""
    from fedbiomed_amd.secagg import SecaggCrypter

    jc = SecaggCrypter()
    for c in n1["crypter"]:
        with caplog.at_level(logging.WARNING):
            got = jc.encrypt(num_nodes=2, current_round=1, params=[F(v) for v in c["x"]], key=I(c["key"]),
                             biprime=1, weight=c["weight"])
        assert got == [I(v) for v in c["enc"]["ok"]]
        _run(c["agg"], lambda: jc.aggregate(current_round=1, num_nodes=2, params=[got, got], key=-I(c["key"]),
                                            biprime=1, total_sample_size=4, num_expected_params=len(c["x"])))


@pytest.mark.gpu
def test_n_one_object_api_gpu(n1):
    """UserKey.encrypt, EncryptedNumber sums, FDH.H, JoyeLibert.protect / aggregate and ServerKey.decrypt
    (an empty list too) at N = 1 against the reference's outcomes."""
    from fedbiomed_amd.secagg._jls import FDH, EncryptedNumber, JoyeLibert, ServerKey, UserKey
    from tests.test_jls_api import pp_of

    o = n1["object"]
    pp = pp_of(1)
    assert UserKey(pp, 3).encrypt([1, 5, 0], 1) == [I(v) for v in o["user_encrypt"]["ok"]]
    assert UserKey(pp, -3).encrypt([1, 5], 2) == [I(v) for v in o["user_encrypt_neg"]["ok"]]
    assert UserKey(pp, 0).encrypt([4], 1) == [I(v) for v in o["user_encrypt_zero_key"]["ok"]]
    s = EncryptedNumber(pp, 0) + EncryptedNumber(pp, 0)
    assert s.ciphertext == I(o["sum"]["ok"])
    assert FDH(2048, 1).H(5) == I(o["fdh"]["ok"])
    _run(o["decrypt"], lambda: ServerKey(pp, -3).decrypt([EncryptedNumber(pp, 0)], 1))
    _run(o["decrypt_empty"], lambda: ServerKey(pp, -3).decrypt([], 1))
    jl = JoyeLibert()
    assert jl.protect(pp, UserKey(pp, 3), 1, [1, 2, 3], 2) == [I(v) for v in o["protect"]["ok"]]
    _run(o["aggregate"], lambda: jl.aggregate(ServerKey(pp, -6), 1, [[EncryptedNumber(pp, 0)]] * 2, 3))


@pytest.mark.gpu
def test_n_one_factor_and_product_gpu():
    """The split entry points at N = 1: the decryption factor and the ciphertext product are 0 (device
    tensors through the C-ABI)."""
    import torch

    from fedbiomed_amd import _device as D

    dev = D.device()
    f = D.jl_decrypt_factor(5, 1, -12345, 1, dev=dev)
    assert not torch.any(f).item()
    rows = torch.zeros((3, 5, 64), dtype=torch.int32, device=dev)
    assert not torch.any(D.jl_product(rows, 1)).item()
    np.testing.assert_array_equal(D.to_host(f).numpy(), 0)
