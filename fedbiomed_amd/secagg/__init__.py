from ._additive_ss import AdditiveSecret, AdditiveShare, AdditiveShares
from ._dh import DHKey, DHKeyAgreement
from ._jls import EncryptedNumber, JoyeLibert
from ._lom import LOM, PRF
from ._secagg_crypter import SecaggCrypter, SecaggLomCrypter

__all__ = ["AdditiveSecret", "AdditiveShare", "AdditiveShares", "DHKey", "DHKeyAgreement", "EncryptedNumber",
           "JoyeLibert", "LOM", "PRF", "SecaggCrypter", "SecaggLomCrypter"]
