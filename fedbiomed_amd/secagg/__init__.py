from ._lom import LOM, PRF
from ._secagg_crypter import SecaggCrypter, SecaggLomCrypter

__all__ = ["LOM", "PRF", "SecaggCrypter", "SecaggLomCrypter"]
