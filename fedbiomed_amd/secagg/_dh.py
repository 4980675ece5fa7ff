"""Setup-time key agreement: ephemeral-ephemeral ECDH on P-256 + ConcatKDF.

Mirror of the reference's `fedbiomed/common/secagg/_dh.py:15-170` (`DHKey`,
`DHKeyAgreement`): same constructors, methods, PEM formats (PKCS#8 private keys,
SubjectPublicKeyInfo public keys), node-id ordering and KDF, same error class and FB629
prefix.  It runs once per experiment and node pair on the host: the elliptic-curve work is
done by the system OpenSSL 3 `libcrypto` through ctypes -- the library the reference's
`cryptography` package drives (cryptography 40.0.2, `pdm.lock:532-533`) -- so the `cryptography`
package is not needed; the ConcatKDF (NIST SP 800-56A single-step KDF, SHA-256) is restated
with hashlib.  Nothing here touches the GPU.  Pinned by `tests/test_dh.py` against vectors the
reference itself produced (`tests/golden/dh.json`, `tools/gen_golden.py`).
"""

import ctypes
import ctypes.util
import hashlib
import threading
from typing import Optional

from ..constants import ErrorNumbers
from ..exceptions import FedbiomedSecaggCrypterError

_lock = threading.Lock()
_lib = None


def _ssl():
    """libcrypto with the prototypes this module uses (loaded on first use)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        lib = ctypes.CDLL(name)
        vp, cp, i, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_size_t
        protos = {
            "EVP_PKEY_CTX_new_from_name": (vp, [vp, cp, cp]),
            "EVP_PKEY_CTX_new": (vp, [vp, vp]),
            "EVP_PKEY_CTX_free": (None, [vp]),
            "EVP_PKEY_keygen_init": (i, [vp]),
            "EVP_PKEY_CTX_set_group_name": (i, [vp, cp]),
            "EVP_PKEY_generate": (i, [vp, ctypes.POINTER(vp)]),
            "EVP_PKEY_free": (None, [vp]),
            "EVP_PKEY_get_base_id": (i, [vp]),
            "EVP_PKEY_derive_init": (i, [vp]),
            "EVP_PKEY_derive_set_peer": (i, [vp, vp]),
            "EVP_PKEY_derive": (i, [vp, ctypes.c_char_p, ctypes.POINTER(sz)]),
            "BIO_new_mem_buf": (vp, [cp, i]),
            "BIO_new": (vp, [vp]),
            "BIO_s_mem": (vp, []),
            "BIO_ctrl": (ctypes.c_long, [vp, i, ctypes.c_long, vp]),
            "BIO_free": (i, [vp]),
            "PEM_read_bio_PrivateKey": (vp, [vp, vp, vp, vp]),
            "PEM_read_bio_PUBKEY": (vp, [vp, vp, vp, vp]),
            "PEM_write_bio_PKCS8PrivateKey": (i, [vp, vp, vp, cp, i, vp, vp]),
            "PEM_write_bio_PUBKEY": (i, [vp, vp]),
            "ERR_clear_error": (None, []),
        }
        for fn, (res, args) in protos.items():
            f = getattr(lib, fn)
            f.restype, f.argtypes = res, args
        _lib = lib
        return lib


_EVP_PKEY_EC = 408  # NID_X9_62_id_ecPublicKey
# pem_password_cb(char *buf, int size, int rwflag, void *u): OpenSSL asks for a pass phrase through
# it; with a NULL callback it would fall back to PEM_def_callback, which prompts on the terminal
_PEM_PASSWORD_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)
_BIO_CTRL_INFO = 3  # BIO_get_mem_data


class _PKey:
    """Owns an OpenSSL EVP_PKEY (an EC key on P-256 when generated here)."""

    def __init__(self, ptr: int, private: bool):
        self._p = ptr
        self.is_private = private

    def __del__(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.EVP_PKEY_free(self._p)
            self._p = None

    def _pem(self, private: bool) -> bytes:
        lib = _ssl()
        bio = lib.BIO_new(lib.BIO_s_mem())
        if not bio:
            raise MemoryError("OpenSSL: no memory BIO")
        try:
            ok = (lib.PEM_write_bio_PKCS8PrivateKey(bio, self._p, None, None, 0, None, None) if private
                  else lib.PEM_write_bio_PUBKEY(bio, self._p))
            if ok != 1:
                raise ValueError("OpenSSL could not serialise the key")
            buf = ctypes.c_void_p()
            n = lib.BIO_ctrl(bio, _BIO_CTRL_INFO, 0, ctypes.byref(buf))
            return ctypes.string_at(buf, n)
        finally:
            lib.BIO_free(bio)

    def public_key(self) -> "_PKey":
        """The public half (a fresh EVP_PKEY read back from its SubjectPublicKeyInfo)."""
        return _load(self._pem(False), private=False)


def _generate_p256() -> _PKey:
    lib = _ssl()
    ctx = lib.EVP_PKEY_CTX_new_from_name(None, b"EC", None)
    if not ctx:
        raise RuntimeError("OpenSSL: no EC key context")
    try:
        pkey = ctypes.c_void_p()
        if (lib.EVP_PKEY_keygen_init(ctx) != 1 or lib.EVP_PKEY_CTX_set_group_name(ctx, b"P-256") != 1
                or lib.EVP_PKEY_generate(ctx, ctypes.byref(pkey)) != 1):
            raise RuntimeError("OpenSSL: P-256 key generation failed")
        return _PKey(pkey.value, private=True)
    finally:
        lib.EVP_PKEY_CTX_free(ctx)


def _load(data: bytes, private: bool) -> _PKey:
    """PEM bytes -> key; ValueError on anything OpenSSL does not parse (as cryptography's
    load_pem_private_key / load_pem_public_key).  An encrypted private key is refused with
    cryptography's TypeError for load_pem_private_key(password=None): the pass-phrase callback
    only records that OpenSSL asked and returns -1, so nothing ever prompts."""
    if not isinstance(data, (bytes, bytearray)):
        raise TypeError("data must be bytes")
    lib = _ssl()
    buf = bytes(data)  # held until the BIO is freed: a memory BIO reads the caller's buffer in place
    bio = lib.BIO_new_mem_buf(buf, len(buf))
    if not bio:
        raise MemoryError("OpenSSL: no memory BIO")
    asked = []

    def no_password(_buf, _size, _rwflag, _u):
        asked.append(True)
        return -1

    cb = _PEM_PASSWORD_CB(no_password)  # alive until the read returns
    try:
        fn = lib.PEM_read_bio_PrivateKey if private else lib.PEM_read_bio_PUBKEY
        p = fn(bio, None, ctypes.cast(cb, ctypes.c_void_p), None)
    finally:
        lib.BIO_free(bio)
        lib.ERR_clear_error()
    if not p:
        if asked:
            raise TypeError("Password was not given but private key is encrypted")
        raise ValueError("Could not deserialize key data.")
    return _PKey(p, private=private)


def _ecdh(priv: _PKey, peer: _PKey) -> bytes:
    """The raw ECDH shared secret (the x coordinate, 32 bytes on P-256), as
    EllipticCurvePrivateKey.exchange(ec.ECDH(), peer) returns it."""
    lib = _ssl()
    if lib.EVP_PKEY_get_base_id(priv._p) != _EVP_PKEY_EC or lib.EVP_PKEY_get_base_id(peer._p) != _EVP_PKEY_EC:
        raise TypeError("ECDH needs elliptic-curve keys")
    ctx = lib.EVP_PKEY_CTX_new(priv._p, None)
    if not ctx:
        raise ValueError("Error computing shared key.")
    try:
        n = ctypes.c_size_t(0)
        if (lib.EVP_PKEY_derive_init(ctx) != 1 or lib.EVP_PKEY_derive_set_peer(ctx, peer._p) != 1
                or lib.EVP_PKEY_derive(ctx, None, ctypes.byref(n)) != 1):
            raise ValueError("Error computing shared key.")
        buf = ctypes.create_string_buffer(n.value)
        if lib.EVP_PKEY_derive(ctx, buf, ctypes.byref(n)) != 1:
            raise ValueError("Error computing shared key.")
        return buf.raw[:n.value]
    finally:
        lib.EVP_PKEY_CTX_free(ctx)
        lib.ERR_clear_error()


def concat_kdf_sha256(z: bytes, length: int, otherinfo: bytes) -> bytes:
    """NIST SP 800-56A single-step KDF with SHA-256 (cryptography's ConcatKDFHash):
    K = H(1 || Z || otherinfo) || H(2 || Z || otherinfo) || ..., counters big-endian 32-bit."""
    out, c = b"", 1
    while len(out) < length:
        out += hashlib.sha256(c.to_bytes(4, "big") + z + otherinfo).digest()
        c += 1
    return out[:length]


class DHKey:
    """P-256 key pair for ephemeral-ephemeral ECDH (reference `_dh.py:15-110`).

    Args:
        private_key_pem: a PEM private key to import (PKCS#8 or traditional), or None.
        public_key_pem: a PEM public key (SubjectPublicKeyInfo) to import, or None.
    With neither, a new P-256 key pair is generated; with only a public key, `private_key`
    is None.
    """

    def __init__(self, private_key_pem: Optional[bytes] = None, public_key_pem: Optional[bytes] = None) -> None:
        if private_key_pem:
            self.private_key = self._import_key(_load, data=private_key_pem, private=True)
        elif not public_key_pem:
            self.private_key = _generate_p256()
        else:
            self.private_key = None
        if public_key_pem:
            self.public_key = self._import_key(_load, data=public_key_pem, private=False)
        else:
            self.public_key = self.private_key.public_key()

    def export_private_key(self) -> Optional[bytes]:
        """PKCS#8 PEM, unencrypted (None without a private key)."""
        if not self.private_key:
            return None
        return self.private_key._pem(True)

    def export_public_key(self) -> bytes:
        """SubjectPublicKeyInfo PEM."""
        return self.public_key._pem(False)

    @staticmethod
    def _import_key(func, **kwargs):
        try:
            return func(**kwargs)
        except ValueError as exp:
            shown = {k: v for k, v in kwargs.items() if k != "private"}
            raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB629.value}: Invalid key format, {shown}") from exp


class DHKeyAgreement:
    """Key agreement of node u with node v (reference `_dh.py:113-170`): ECDH shared secret,
    then a 32-byte ConcatKDF-SHA256 key with otherinfo = session_salt || the two node ids in
    ascending (Python string) order."""

    def __init__(self, node_u_id, node_u_dh_key: DHKey, session_salt):
        self._node_u_id = node_u_id
        self._dh_key = node_u_dh_key
        self.session_salt = session_salt

    def _kdf(self, key, node_v_id):
        node_ids = self._node_u_id + node_v_id if self._node_u_id < node_v_id else node_v_id + self._node_u_id
        return concat_kdf_sha256(key, 32, self.session_salt + node_ids.encode("utf-8"))

    def agree(self, node_v_id, public_key_pem):
        dh_v_key = DHKey(public_key_pem=public_key_pem)
        shared_secret = _ecdh(self._dh_key.private_key, dh_v_key.public_key)
        return self._kdf(shared_secret, node_v_id)
