"""Setup-time key agreement: fedbiomed_amd.secagg.DHKey / DHKeyAgreement
against vectors the reference itself produced (tests/golden/dh.json, tools/gen_golden.py:
fedbiomed/common/secagg/_dh.py run through tools/refshim) -- byte-identical PEM exports of the
reference's keys, the pairwise keys its agreement derives (ECDH P-256 + ConcatKDF-SHA256 over
salt || ordered ids) for every ordered pair of six ids under three salts, its _kdf on fixed
secrets and its error outcomes -- plus the reference's own test behaviours (tests/test_dh.py).
Host only: no GPU."""

import pytest

from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError
from fedbiomed_amd.secagg import DHKey, DHKeyAgreement
from fedbiomed_amd.secagg._dh import concat_kdf_sha256


@pytest.fixture(scope="module")
def dh(golden):
    return golden["dh"]


def test_pem_roundtrip_is_byte_identical(dh):
    for priv, pub in zip(dh["private_pem"], dh["public_pem"]):
        k = DHKey(private_key_pem=priv.encode())
        assert k.export_private_key() == priv.encode()
        assert k.export_public_key() == pub.encode()
        assert DHKey(public_key_pem=pub.encode()).export_public_key() == pub.encode()


def test_pairwise_keys_match_reference(dh):
    ids, priv, pub = dh["ids"], dh["private_pem"], dh["public_pem"]
    keys = [DHKey(private_key_pem=p.encode()) for p in priv]
    for c in dh["pairs"]:
        ka = DHKeyAgreement(ids[c["u"]], keys[c["u"]], bytes.fromhex(c["salt"]))
        assert ka.agree(ids[c["v"]], pub[c["v"]].encode()).hex() == c["key"], c


def test_kdf_matches_reference(dh):
    k0 = DHKey(private_key_pem=dh["private_pem"][0].encode())
    for c in dh["kdf"]:
        ka = DHKeyAgreement(c["u"], k0, bytes.fromhex(c["salt"]))
        assert ka._kdf(bytes.fromhex(c["secret"]), c["v"]).hex() == c["key"]


def test_error_outcomes_match_reference(dh):
    errs = dh["errors"]
    assert errs["bad_private"]["error"] == "FedbiomedSecaggCrypterError"
    assert errs["bad_public"]["error"] == "FedbiomedSecaggCrypterError"
    assert errs["private_as_public"]["error"] == "FedbiomedSecaggCrypterError"
    assert errs["public_only_export_private"] == {"ok": None}
    for kw in ({"private_key_pem": b"invalid_key_data"}, {"public_key_pem": b"invalid_key_data"}):
        with pytest.raises(FedbiomedSecaggCrypterError, match="FB629"):
            DHKey(**kw)
    k = DHKey()
    with pytest.raises(FedbiomedSecaggCrypterError, match="FB629"):
        DHKeyAgreement("u", k, b"s").agree("v", k.export_private_key())
    assert DHKey(public_key_pem=dh["public_pem"][0].encode()).export_private_key() is None


def test_fresh_keys_agree_both_ways():
    """The reference's test_dh.py behaviours on freshly generated P-256 keys."""
    u, v = DHKey(), DHKey()
    assert isinstance(u.export_private_key(), bytes) and isinstance(u.export_public_key(), bytes)
    assert u.export_private_key().startswith(b"-----BEGIN PRIVATE KEY-----")
    assert u.export_public_key().startswith(b"-----BEGIN PUBLIC KEY-----")
    a_u = DHKeyAgreement("node_u", DHKey(u.export_private_key()), b"this_is_a_salt")
    a_v = DHKeyAgreement("node_v", DHKey(v.export_private_key()), b"this_is_a_salt")
    k_uv, k_vu = a_u.agree("node_v", v.export_public_key()), a_v.agree("node_u", u.export_public_key())
    assert k_uv == k_vu and len(k_uv) == 32
    assert len(a_u._kdf(b"secret_key", "node_v")) == 32
    assert DHKey().export_public_key() != u.export_public_key()  # fresh randomness


def test_concat_kdf_multi_block():
    """Outputs longer than one SHA-256 block chain the 32-bit big-endian counter (SP 800-56A)."""
    import hashlib

    z, info = b"\x01" * 32, b"info"
    out = concat_kdf_sha256(z, 70, info)
    want = b"".join(hashlib.sha256(c.to_bytes(4, "big") + z + info).digest() for c in (1, 2, 3))[:70]
    assert out == want


def test_bytearray_pem_input(dh):
    """PEM handed over as a bytearray (a temporary bytes copy must outlive OpenSSL's memory BIO)."""
    import gc

    priv, pub = dh["private_pem"][1].encode(), dh["public_pem"][1].encode()
    for _ in range(20):
        k = DHKey(private_key_pem=bytearray(priv))
        gc.collect()
        assert k.export_public_key() == pub
        assert DHKey(public_key_pem=bytearray(pub)).export_public_key() == pub


def test_encrypted_private_pem_is_refused_without_prompting():
    """An encrypted PKCS#8 PEM with no password: cryptography's load_pem_private_key(password=None)
    raises TypeError (the reference's _import_key lets it through); OpenSSL must not fall back to
    its terminal prompt (PEM_def_callback)."""
    import ctypes

    from fedbiomed_amd.secagg import _dh

    lib = _dh._ssl()
    lib.EVP_aes_256_cbc.restype = ctypes.c_void_p
    k = DHKey()
    bio = lib.BIO_new(lib.BIO_s_mem())
    try:
        assert lib.PEM_write_bio_PKCS8PrivateKey(bio, k.private_key._p, lib.EVP_aes_256_cbc(), b"pw", 2, None,
                                                 None) == 1
        buf = ctypes.c_void_p()
        n = lib.BIO_ctrl(bio, 3, 0, ctypes.byref(buf))
        pem = ctypes.string_at(buf, n)
    finally:
        lib.BIO_free(bio)
    assert b"ENCRYPTED PRIVATE KEY" in pem
    with pytest.raises(TypeError, match="Password was not given but private key is encrypted"):
        DHKey(private_key_pem=pem)
