"""ChaCha20 known-answer tests (RFC 7539 §2.3.2 block function, §2.4.2 encryption) for the
three ChaCha20s of the LOM path: the oracle's numpy restatement, the refshim stand-in for
`cryptography` (OpenSSL EVP_chacha20, what the reference's `_lom.py:43-47,70-72` calls), and
the HIP keystream (through `fbm_prf_key`, `-m gpu`).  OpenSSL reads the 16-byte IV as a
64-bit little-endian block counter (bytes 0-7, carrying from word 12 into word 13) and an
8-byte nonce; the carry cases pin that convention.
"""

import os
import sys

import numpy as np
import pytest

from oracle import secagg_oracle as O

KEY = bytes(range(32))
# RFC 7539 §2.3.2: counter 1, nonce 00000009 0000004a 00000000 -> serialized block
IV_232 = (1).to_bytes(4, "little") + bytes.fromhex("000000090000004a00000000")
BLOCK_232 = bytes.fromhex("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                          "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")
# RFC 7539 §2.4.2: counter 1, nonce 00000000 0000004a 00000000, the "sunscreen" plaintext
IV_242 = (1).to_bytes(4, "little") + bytes.fromhex("000000000000004a00000000")
PT_242 = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, "
          b"sunscreen would be it.")
CT_242 = bytes.fromhex("6e2e359a2568f98041ba0728dd0d6981e97e7aec1d4360c20a27afccfd9fae0bf91b65c5524733ab8f593dab"
                       "cd62b3571639d624e65152ab8f530c359f0861d807ca0dbf500d6a6156a38e088a22b65e52bc514d16ccf80681"
                       "8ce91ab77937365af90bbf74a35be6b40b8eedf2785e42874d")
# counter words 12-13 right below a 32-bit and a 64-bit wrap
CARRY_IVS = [bytes.fromhex("feffffff05000000") + bytes(range(8)),
             bytes.fromhex("ffffffff00000000") + b"\xaa" * 8,
             bytes.fromhex("feffffffffffffff") + b"\x01" * 8]


def _xor(a, b):
    return bytes(x ^ y for x, y in zip(a, b))


def _refshim():
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "refshim")
    if not os.path.isdir(here):
        pytest.skip("tools/refshim not present (it does not travel to the GPU box)")
    sys.path.insert(0, here)
    try:
        from cryptography.hazmat.primitives.ciphers import Cipher, algorithms
    except OSError:
        pytest.skip("libcrypto not loadable")
    finally:
        sys.path.remove(here)
    return lambda key, iv, data: Cipher(algorithms.ChaCha20(key, iv)).encryptor().update(data)


def test_oracle_rfc7539_block():
    assert O.chacha20_keystream(KEY, IV_232, 64) == BLOCK_232


def test_oracle_rfc7539_encrypt():
    assert _xor(PT_242, O.chacha20_keystream(KEY, IV_242, len(PT_242))) == CT_242


def test_refshim_rfc7539():
    enc = _refshim()
    assert enc(KEY, IV_232, bytes(64)) == BLOCK_232
    assert enc(KEY, IV_242, PT_242) == CT_242


@pytest.mark.parametrize("iv", CARRY_IVS)
def test_counter_carry_oracle_vs_openssl(iv):
    """Blocks straddling the 32-bit (and the 64-bit) counter wrap: the oracle's numpy
    restatement against OpenSSL itself."""
    enc = _refshim()
    ks_ossl = enc(KEY, iv, bytes(64 * 5))
    assert O.chacha20_keystream(KEY, iv, 64 * 5) == ks_ossl
    # block-indexed access (what element-range shards use) agrees with the stream
    blk = O.chacha20_blocks(KEY, iv, 3, 2).astype("<u4").tobytes()
    assert blk == ks_ossl[3 * 64:5 * 64]


@pytest.mark.gpu
def test_device_keystream_rfc7539_and_carry():
    """The HIP ChaCha20 (PRF.eval_key path: first 16 keystream bytes XOR tau, tau = 0) on the
    RFC vector and on IVs whose counter word carries."""
    from fedbiomed_amd import _device as D

    assert D.prf_key(KEY, IV_232, 0)[:16] == BLOCK_232[:16]
    assert D.prf_key(KEY, IV_242, 0)[:16] == O.chacha20_keystream(KEY, IV_242, 16)
    for iv in CARRY_IVS:
        assert D.prf_key(KEY, iv, 0)[:16] == O.chacha20_keystream(KEY, iv, 16)
    # PRF.eval_vector over a counter wrap: raw-seed LOM protect of zeros with one "peer"
    import torch

    iv = CARRY_IVS[0]
    n = 64
    y = D.lom_protect(torch.zeros(n, dtype=torch.int64, device=D.device()), [KEY], [1], iv, 0, 2,
                      raw_seeds=True)
    want = O.prf_eval_vector(KEY, iv, 0, n)
    assert np.array_equal(y.cpu().numpy().view(np.uint64), want)
