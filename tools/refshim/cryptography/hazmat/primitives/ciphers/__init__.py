"""Stand-in for `cryptography.hazmat.primitives.ciphers` (cryptography 40.0.2 pinned in the
reference's pdm.lock), restricted to `Cipher(algorithms.ChaCha20(key, nonce), mode=None)`
as used by the reference LOM PRF (`fedbiomed/common/secagg/_lom.py:43-47,70-72`).

Backed by the system OpenSSL 3 `EVP_chacha20` through ctypes -- the same library the
real `cryptography` wheel calls -- so the 16-byte nonce is interpreted OpenSSL's way
(bytes 0-7 = 64-bit little-endian block counter with carry, bytes 8-15 = nonce).
Test tooling only; never imported by `fedbiomed_amd`.
"""

import ctypes
import ctypes.util

_ssl = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
_ssl.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_ssl.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
_ssl.EVP_chacha20.restype = ctypes.c_void_p
_ssl.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_char_p, ctypes.c_char_p]
_ssl.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                   ctypes.c_char_p, ctypes.c_int]


class algorithms:  # noqa: N801
    class ChaCha20:
        name = "ChaCha20"
        key_size = 256

        def __init__(self, key: bytes, nonce: bytes):
            if not isinstance(key, (bytes, bytearray)) or len(key) != 32:
                raise ValueError("Invalid key size (%s) for ChaCha20." % (len(key) * 8,))
            if not isinstance(nonce, (bytes, bytearray)) or len(nonce) != 16:
                raise ValueError("nonce must be 128-bits (16 bytes)")
            self.key = bytes(key)
            self.nonce = bytes(nonce)


class _Encryptor:
    def __init__(self, alg):
        self._ctx = _ssl.EVP_CIPHER_CTX_new()
        ok = _ssl.EVP_EncryptInit_ex(self._ctx, _ssl.EVP_chacha20(), None, alg.key, alg.nonce)
        if ok != 1:
            raise ValueError("EVP_EncryptInit_ex failed")

    def update(self, data: bytes) -> bytes:
        data = bytes(data)
        out = ctypes.create_string_buffer(len(data) + 64)
        outl = ctypes.c_int(0)
        pos = 0
        chunk = 1 << 30
        res = []
        while pos < len(data) or (pos == 0 and not data):
            part = data[pos:pos + chunk]
            if len(part) > len(out):
                out = ctypes.create_string_buffer(len(part) + 64)
            if _ssl.EVP_EncryptUpdate(self._ctx, out, ctypes.byref(outl), part, len(part)) != 1:
                raise ValueError("EVP_EncryptUpdate failed")
            res.append(out.raw[: outl.value])
            pos += len(part)
            if not data:
                break
        return b"".join(res)

    def finalize(self) -> bytes:
        if self._ctx:
            _ssl.EVP_CIPHER_CTX_free(self._ctx)
            self._ctx = None
        return b""


class Cipher:
    def __init__(self, algorithm, mode=None, backend=None):
        self.algorithm = algorithm

    def encryptor(self):
        return _Encryptor(self.algorithm)
