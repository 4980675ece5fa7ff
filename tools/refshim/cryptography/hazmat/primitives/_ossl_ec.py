"""OpenSSL 3 libcrypto (ctypes) backing for the `cryptography` stand-ins used by the
reference's `fedbiomed/common/secagg/_dh.py`: EC P-256 keys, PEM, ECDH and the SSKDF
(ConcatKDF) -- the library the real `cryptography` 40.0.2 wheel calls.  Test tooling only
(`tools/gen_golden.py`); never imported by `fedbiomed_amd`."""

import ctypes
import ctypes.util

L = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
vp, cp, i, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_size_t


class OSSL_PARAM(ctypes.Structure):  # noqa: N801
    _fields_ = [("key", cp), ("data_type", ctypes.c_uint), ("data", vp), ("data_size", sz), ("return_size", sz)]


for fn, res, args in (
        ("EVP_PKEY_CTX_new_from_name", vp, [vp, cp, cp]), ("EVP_PKEY_CTX_new", vp, [vp, vp]),
        ("EVP_PKEY_CTX_free", None, [vp]), ("EVP_PKEY_keygen_init", i, [vp]),
        ("EVP_PKEY_CTX_set_group_name", i, [vp, cp]), ("EVP_PKEY_generate", i, [vp, ctypes.POINTER(vp)]),
        ("EVP_PKEY_derive_init", i, [vp]), ("EVP_PKEY_derive_set_peer", i, [vp, vp]),
        ("EVP_PKEY_derive", i, [vp, cp, ctypes.POINTER(sz)]), ("BIO_new_mem_buf", vp, [cp, i]),
        ("BIO_new", vp, [vp]), ("BIO_s_mem", vp, []), ("BIO_ctrl", ctypes.c_long, [vp, i, ctypes.c_long, vp]),
        ("BIO_free", i, [vp]), ("PEM_read_bio_PrivateKey", vp, [vp, vp, vp, vp]),
        ("PEM_read_bio_PUBKEY", vp, [vp, vp, vp, vp]), ("PEM_write_bio_PKCS8PrivateKey", i, [vp, vp, vp, cp, i, vp, vp]),
        ("PEM_write_bio_PUBKEY", i, [vp, vp]), ("EVP_PKEY_get_base_id", i, [vp]),
        ("EVP_KDF_fetch", vp, [vp, cp, cp]), ("EVP_KDF_CTX_new", vp, [vp]), ("EVP_KDF_CTX_free", None, [vp]),
        ("EVP_KDF_free", None, [vp]), ("EVP_KDF_derive", i, [vp, cp, sz, ctypes.POINTER(OSSL_PARAM)]),
        ("OSSL_PARAM_construct_utf8_string", OSSL_PARAM, [cp, cp, sz]),
        ("OSSL_PARAM_construct_octet_string", OSSL_PARAM, [cp, vp, sz]),
        ("OSSL_PARAM_construct_end", OSSL_PARAM, []), ("ERR_clear_error", None, [])):
    f = getattr(L, fn)
    f.restype, f.argtypes = res, args


def generate_p256():
    ctx = L.EVP_PKEY_CTX_new_from_name(None, b"EC", None)
    p = vp()
    assert L.EVP_PKEY_keygen_init(ctx) == 1 and L.EVP_PKEY_CTX_set_group_name(ctx, b"P-256") == 1
    assert L.EVP_PKEY_generate(ctx, ctypes.byref(p)) == 1
    L.EVP_PKEY_CTX_free(ctx)
    return p.value


def read_pem(data: bytes, private: bool):
    bio = L.BIO_new_mem_buf(bytes(data), len(data))
    p = (L.PEM_read_bio_PrivateKey if private else L.PEM_read_bio_PUBKEY)(bio, None, None, None)
    L.BIO_free(bio)
    L.ERR_clear_error()
    if not p:
        raise ValueError("Could not deserialize key data.")
    return p


def write_pem(p, private: bool) -> bytes:
    bio = L.BIO_new(L.BIO_s_mem())
    ok = L.PEM_write_bio_PKCS8PrivateKey(bio, p, None, None, 0, None, None) if private else L.PEM_write_bio_PUBKEY(bio, p)
    assert ok == 1
    buf = vp()
    n = L.BIO_ctrl(bio, 3, 0, ctypes.byref(buf))
    out = ctypes.string_at(buf, n)
    L.BIO_free(bio)
    return out


def is_ec(p) -> bool:
    return L.EVP_PKEY_get_base_id(p) == 408


def derive(p, peer) -> bytes:
    ctx = L.EVP_PKEY_CTX_new(p, None)
    n = sz(0)
    ok = L.EVP_PKEY_derive_init(ctx) == 1 and L.EVP_PKEY_derive_set_peer(ctx, peer) == 1 and \
        L.EVP_PKEY_derive(ctx, None, ctypes.byref(n)) == 1
    buf = ctypes.create_string_buffer(max(1, n.value))
    ok = ok and L.EVP_PKEY_derive(ctx, buf, ctypes.byref(n)) == 1
    L.EVP_PKEY_CTX_free(ctx)
    L.ERR_clear_error()
    if not ok:
        raise ValueError("Error computing shared key.")
    return buf.raw[:n.value]


def sskdf_sha256(key: bytes, length: int, info: bytes) -> bytes:
    """OpenSSL's single-step KDF (SP 800-56C rev. 2 = ConcatKDF) with SHA-256."""
    kdf = L.EVP_KDF_fetch(None, b"SSKDF", None)
    ctx = L.EVP_KDF_CTX_new(kdf)
    kb, ib = ctypes.create_string_buffer(key, len(key)), ctypes.create_string_buffer(info, max(1, len(info)))
    params = (OSSL_PARAM * 4)(L.OSSL_PARAM_construct_utf8_string(b"digest", b"SHA256", 0),
                              L.OSSL_PARAM_construct_octet_string(b"key", ctypes.cast(kb, vp), len(key)),
                              L.OSSL_PARAM_construct_octet_string(b"info", ctypes.cast(ib, vp), len(info)),
                              L.OSSL_PARAM_construct_end())
    out = ctypes.create_string_buffer(length)
    ok = L.EVP_KDF_derive(ctx, out, length, params)
    L.EVP_KDF_CTX_free(ctx)
    L.EVP_KDF_free(kdf)
    assert ok == 1, "SSKDF failed"
    return out.raw
