"""Stand-in for `cryptography.hazmat.primitives.kdf.concatkdf.ConcatKDFHash` (SHA-256), the
reference's pairwise-key KDF (`fedbiomed/common/secagg/_dh.py:146-152`), backed by OpenSSL's
SSKDF (SP 800-56C single-step KDF == ConcatKDF).  Test tooling only."""

from .. import _ossl_ec as O


class ConcatKDFHash:
    def __init__(self, algorithm, length, otherinfo, backend=None):
        if getattr(algorithm, "name", None) != "sha256":
            raise NotImplementedError("only SHA256 is shimmed")
        if otherinfo is not None and not isinstance(otherinfo, (bytes, bytearray)):
            raise TypeError("otherinfo must be bytes.")
        self._len, self._info, self._used = length, bytes(otherinfo or b""), False

    def derive(self, key_material):
        if self._used:
            raise RuntimeError("AlreadyFinalized")
        self._used = True
        return O.sskdf_sha256(bytes(key_material), self._len, self._info)
