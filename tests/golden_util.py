"""Decoding helpers for the committed golden fixtures (tests/golden/*.json).

Fixtures are data produced by the reference implementation (tools/gen_golden.py):
big ints are "0x.." hex strings, float64 values "f:<16 hex digits>" IEEE bit patterns.
"""

import json
import os
import struct

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def I(s):  # noqa: E743
    return int(s, 16)


def F(s):
    assert s.startswith("f:")
    return struct.unpack(">d", bytes.fromhex(s[2:]))[0]


def fbits(x: float) -> str:
    return struct.pack(">d", float(x)).hex()


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_all():
    return {k: load(k + ".json") for k in ("quantize", "lom", "jl", "ass", "edge", "dh", "jls_api", "crypter_sweep", "even",
                                           "api_edges", "custom_hash", "ass_stream")}


def custom_hashes():
    """Hashing functions other than FBM's FDH(2048, N^2).H, the same callables for the reference run
    that made tests/golden/custom_hash.json (tools/gen_golden.py gen_custom_hash) and for the tests:
    a small affine map, one past 2^2048 (reduced mod N^2 by powmod), a negative one, a SHA-256 based
    2048-bit one and the constant 1 (powmod's shortcut)."""
    import hashlib

    def sha(t):
        return int.from_bytes(hashlib.sha256(int(t).to_bytes(128, "big")).digest() * 8, "big")

    return {
        "affine": lambda t: 5 * int(t) + 3,
        "wide": lambda t: (int(t) * 0x9E3779B97F4A7C15 + 1) ** 4 + 11,
        "negative": lambda t: -(int(t) + 2),
        "sha": sha,
        "one": lambda t: 1,
    }
