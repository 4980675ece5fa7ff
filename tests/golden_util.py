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
                                           "api_edges")}
