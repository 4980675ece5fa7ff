"""Stand-in for `cryptography.hazmat.primitives.serialization` as the reference's
`_dh.py:38-92` uses it (PEM, PKCS#8 / SubjectPublicKeyInfo, NoEncryption, PEM loaders),
backed by OpenSSL (`_ossl_ec`).  Test tooling only."""

import enum

from . import _ossl_ec as O


class Encoding(enum.Enum):
    PEM = "PEM"


class PrivateFormat(enum.Enum):
    PKCS8 = "PKCS8"


class PublicFormat(enum.Enum):
    SubjectPublicKeyInfo = "X.509 subjectPublicKeyInfo with PKCS#1"


class NoEncryption:
    pass


def load_pem_private_key(data, password=None, backend=None, **kw):
    from .asymmetric.ec import EllipticCurvePrivateKey

    if password is not None:
        raise TypeError("Password was given but private key is not encrypted.")
    return EllipticCurvePrivateKey(O.read_pem(data, True))


def load_pem_public_key(data, backend=None):
    from .asymmetric.ec import EllipticCurvePublicKey

    return EllipticCurvePublicKey(O.read_pem(data, False))
