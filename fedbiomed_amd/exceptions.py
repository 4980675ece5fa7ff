"""Exception hierarchy mirrored from the reference (fedbiomed/common/exceptions.py:10,209,217,290,306)
so callers' `except` clauses keep working."""


class FedbiomedError(Exception):
    """Top class of all Fed-BioMed exceptions."""


class FedbiomedSecaggError(FedbiomedError):
    """Secure aggregation error (FB417)."""


class FedbiomedSecaggCrypterError(FedbiomedError):
    """Secure aggregation crypter error (FB624)."""


class FedbiomedTypeError(FedbiomedError, TypeError):
    """TypeError for Fed-BioMed."""


class FedbiomedValueError(FedbiomedError, ValueError):
    """ValueError for Fed-BioMed."""
