"""Stand-in for `cryptography.hazmat.primitives.asymmetric.ec` (P-256 keys, ECDH) as the
reference's `_dh.py` and `tests/test_dh.py` use it, backed by OpenSSL (`_ossl_ec`).
Test tooling only."""

from .. import _ossl_ec as O
from ..serialization import Encoding, PrivateFormat, PublicFormat


class SECP256R1:
    name = "secp256r1"
    key_size = 256


class ECDH:
    pass


class EllipticCurvePublicKey:
    def __init__(self, p):
        if not O.is_ec(p):
            raise ValueError("not an EC key")
        self._p = p

    def public_bytes(self, encoding, format):
        assert encoding == Encoding.PEM and format == PublicFormat.SubjectPublicKeyInfo
        return O.write_pem(self._p, False)


class EllipticCurvePrivateKey:
    def __init__(self, p):
        if not O.is_ec(p):
            raise ValueError("not an EC key")
        self._p = p

    def public_key(self):
        return EllipticCurvePublicKey(O.read_pem(O.write_pem(self._p, False), False))

    def private_bytes(self, encoding, format, encryption_algorithm):
        assert encoding == Encoding.PEM and format == PrivateFormat.PKCS8
        return O.write_pem(self._p, True)

    def exchange(self, algorithm, peer_public_key):
        assert isinstance(algorithm, ECDH)
        return O.derive(self._p, peer_public_key._p)


def generate_private_key(curve, backend=None):
    assert isinstance(curve, SECP256R1)
    return EllipticCurvePrivateKey(O.generate_p256())
