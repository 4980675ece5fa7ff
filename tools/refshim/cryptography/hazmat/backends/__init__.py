"""Stand-in for `cryptography.hazmat.backends` (test tooling only, see tools/refshim/gmpy2)."""


def default_backend():
    return None
