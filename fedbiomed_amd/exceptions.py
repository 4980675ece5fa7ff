"""The reference's exception classes (fedbiomed/common/exceptions.py:10,209,217,290,306).

When Fed-BioMed itself is importable (the drop-in runs inside a node or a researcher), the names
below ARE `fedbiomed.common.exceptions`' classes, bound here before any other module of this
package imports them: the crypters then raise exactly what the reference raises, and the
researcher's `except FedbiomedError` (researcher/federated_workflows/_federated_workflow.py:94)
catches them.  Without Fed-BioMed (stand-alone use, the GPU test box) the same names are mirrors
with the reference's hierarchy.  `BOUND_TO_REFERENCE` says which one is in force.
"""

try:  # the reference module imports nothing else from fedbiomed (its own header says so)
    from fedbiomed.common.exceptions import (  # type: ignore[import-not-found]
        FedbiomedError,
        FedbiomedSecaggCrypterError,
        FedbiomedSecaggError,
        FedbiomedTypeError,
        FedbiomedValueError,
    )

    BOUND_TO_REFERENCE = True
except ImportError:
    BOUND_TO_REFERENCE = False

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


__all__ = [
    "BOUND_TO_REFERENCE",
    "FedbiomedError",
    "FedbiomedSecaggError",
    "FedbiomedSecaggCrypterError",
    "FedbiomedTypeError",
    "FedbiomedValueError",
]
