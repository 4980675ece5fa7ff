"""Stand-in for `cryptography.hazmat.primitives.hashes` (SHA256 only: the reference's
ConcatKDFHash, `fedbiomed/common/secagg/_dh.py:146-151`).  Test tooling only."""


class SHA256:
    name = "sha256"
    digest_size = 32
    block_size = 64
