"""The 74-limb Montgomery product of the combine kernels (tools/gen_mont_asm.py -> csrc/fbm_mont_asm.hpp),
interpreted instruction by instruction on the CPU (tests/asm_sim.py) against Python integers.

Round 6: `fbm_mm_row` takes its B operand from the lane's 64-word ciphertext row in global memory and
converts it to 28-bit limbs in B's registers (no LDS staging column: `jl_prod_kernel` / `jl_encf_kernel` then
need half the LDS and run two waves per SIMD).  It must equal the LDS-column form bit for bit: a * b * R^-1
mod M, lazily reduced (< 2M), R = 2^2072, for every b < 2^2048 -- the top limb's 4 bits, words straddling
limbs, b = 0 and b = 2^2048 - 1 included.
"""

import importlib.util
import os
import random

import pytest

from tests.asm_sim import Lane

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NL, LB = 74, 28
R = 1 << (NL * LB)


@pytest.fixture(scope="module")
def gen():
    spec = importlib.util.spec_from_file_location("gen_mont_asm", os.path.join(ROOT, "tools", "gen_mont_asm.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g


def limbs28(v, n=NL):
    return [(v >> (LB * k)) & ((1 << LB) - 1) for k in range(n)]


def run_product(g, bsrc, a, b, M):
    mp = (-pow(M, -1, 1 << LB)) % (1 << LB)
    a_off, b_off, m_base, row = 0x100, 0x200, 0x1000, 0x8000
    lds, glb, smem = {}, {}, {}
    for k, v in enumerate(limbs28(a)):
        lds[a_off + 1024 * k] = v
    for k, v in enumerate(limbs28(M)):
        smem[m_base + 4 * k] = v
    if bsrc == "lds":
        for k, v in enumerate(limbs28(b)):
            lds[b_off + 1024 * k] = v
    else:
        for i in range(64):
            glb[row + 4 * i] = (b >> (32 * i)) & 0xFFFFFFFF
    lane = Lane({"a": a_off, "b": b_off, "r": row, "M": m_base, "mp": mp}, lds=lds, glb=glb, smem=smem)
    lane.run(g.product(bsrc))
    return sum(lds[a_off + 1024 * k] << (LB * k) for k in range(NL))


@pytest.mark.parametrize("seed", range(4))
def test_row_product_equals_lds_product(gen, seed):
    rng = random.Random(600 + seed)
    n = rng.getrandbits(1024) | (1 << 1023) | 1
    M = n * n
    cases = [rng.randrange(M) for _ in range(3)] + [0, 1, (1 << 2048) - 1 if seed % 2 else M - 1,
                                                     sum(0xF << (28 * k + 24) for k in range(73)) % (1 << 2048)]
    a = rng.randrange(2 * M)  # the running product: lazily reduced, < 2M
    for b in cases:
        got = run_product(gen, "row", a, b, M)
        want = run_product(gen, "lds", a, b, M)
        assert got == want, hex(b)
        assert got < 2 * M and got % M == a * b * pow(R, -1, M) % M


def test_row_conversion_is_in_place_safe(gen):
    """The in-place 32 -> 28-bit conversion reads every word before a higher limb overwrites its register:
    checked on the instruction list (register of limb k is never read after it is written)."""
    conv = gen.convert_b_row()
    written = set()
    for ln in conv:
        op, _, rest = ln.partition(" ")
        ops = [t.strip() for t in rest.split(",")]
        srcs = [o for o in ops[1:] if o.startswith("v")]
        dst = ops[0]
        assert not (set(srcs) - {dst}) & written, ln
        written.add(dst)
    assert len(written) == NL
