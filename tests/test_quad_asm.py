"""The generated QUAD N-adic assembly product (fedbiomed_amd/csrc/fbm_quad_asm.hpp, from
tools/gen_quad_asm.py: four lanes per ciphertext, 29-bit limbs, DPP quad_perm exchanges),
run in lockstep for whole quads on the CPU (tests/asm_sim.py Wave) against Python integers:
X*Y*R^-1 mod N^2 with R = 2^1044, digits < 2N, lazy limbs within the documented bound, and
no 64-bit column overflow (asserted by the simulator on every v_mad_u64_u32 -- the point of
the mid-product reduction).  The residues are the one-lane engine's (tests/test_nadic_asm.py);
the GPU tests compare the two engines' canonical outputs bit for bit."""

import importlib.util
import os
import random

import pytest

from tests.asm_sim import Lane, Wave

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


Q = _load("gen_quad_asm")
LB, L, ML, ROWB, D1 = Q.LB, Q.L, Q.M, Q.ROWB, Q.D1
MASK = (1 << LB) - 1
R = 1 << (LB * L)
QMM, QSQ = Q.product(False), Q.product(True)


def limbs(x, n=L):
    return [(x >> (LB * k)) & MASK for k in range(n)]


def qconsts(N):
    """The quad constants the library builds on the host: K'_i = 2^29 - 1 + K_i with
    K = (1 - R) mod N (words 0..35 of the block), np = -N^-1 mod 2^29."""
    K = (1 - R) % N
    return [MASK + v for v in limbs(K)], (-pow(N, -1, 1 << LB)) % (1 << LB)


def run_quad(N, As, Bs=None, lazy_in=False):
    """As / Bs: lists (one per ciphertext = quad) of digit pairs; Bs None = square.
    Returns per ciphertext the result digit integers (t, s), the max limb and the counts."""
    kp, np_ = qconsts(N)
    QK, BB = 0x4000, 0x100000
    smem = {QK + 4 * i: w for i, w in enumerate(kp)}
    lds, glb = {}, {}
    nl = limbs(N)
    lanes = []
    for c in range(len(As)):
        ac = 4 * c
        col = limbs(As[c][0]) + limbs(As[c][1])
        if lazy_in:  # one unit of 2^29 moved from limb 10 into limb 9 of each digit (lazy limbs)
            for d in (0, D1):
                if col[d + 10] > 0:
                    col[d + 10] -= 1
                    col[d + 9] += 1 << LB
        for k, v in enumerate(col):
            lds[ac + k * ROWB] = v
        for l in range(4):
            tid = 4 * c + l
            if Bs is not None:
                bl, bh = limbs(Bs[c][0]), limbs(Bs[c][1])
                for r in range(ML):
                    glb[BB + tid * 4 + r * 1024] = bl[ML * l + r]
                    glb[BB + tid * 4 + (ML + r) * 1024] = bh[ML * l + r]
            args = {"ac": ac, "al": ac + ML * l * ROWB, "b": tid * 4, "bb": BB, "QK": QK, "np": np_,
                    "e0": 1 if l == 0 else 0}
            for r in range(ML):
                args[f"n{r}"] = nl[ML * l + r]
            lanes.append(Lane(args, lds=lds, glb=glb, smem=smem))
    counts = Wave(lanes).run(QMM if Bs is not None else QSQ)
    out, top = [], 0
    for c in range(len(As)):
        col = [lds[4 * c + k * ROWB] for k in range(2 * L)]
        top = max(top, max(col))
        d0 = sum(v << (LB * k) for k, v in enumerate(col[:L]))
        d1 = sum(v << (LB * k) for k, v in enumerate(col[L:]))
        out.append((d0, d1))
    return out, top, counts


def _rand_n(rng, bits):
    return rng.getrandbits(bits) | (1 << (bits - 1)) | 1


@pytest.mark.parametrize("bits", [2, 24, 1024])
def test_quad_product_and_square(bits):
    rng = random.Random(100 + bits)
    N = _rand_n(rng, bits)
    M = N * N
    rinv = pow(R, -1, M)
    As = [(2 * N - 1, 2 * N - 1)] + [(rng.randrange(2 * N), rng.randrange(2 * N)) for _ in range(2)]
    Bs = [(2 * N - 1, 2 * N - 1)] + [(rng.randrange(2 * N), rng.randrange(2 * N)) for _ in range(2)]
    got, top, counts = run_quad(N, As, Bs)
    assert top < (1 << LB) + (1 << 11)
    assert counts["v_mad_u64_u32"] == Q.product_mads(False)
    for a, b, (t, s) in zip(As, Bs, got):
        A, B = (a[0] + a[1] * N) % M, (b[0] + b[1] * N) % M
        assert (t + s * N) % M == A * B * rinv % M
        assert t < 2 * N and s < 2 * N
    got, top, counts = run_quad(N, As)
    assert counts["v_mad_u64_u32"] == Q.product_mads(True)
    for a, (t, s) in zip(As, got):
        A = (a[0] + a[1] * N) % M
        assert (t + s * N) % M == A * A * rinv % M
        assert t < 2 * N and s < 2 * N


def test_quad_worst_case_columns():
    """All-ones limbs (every operand limb 2^29 - 1, and lazy ones above it): the largest column
    sums the bound allows; the simulator's overflow asserts are the check."""
    N = (1 << 1024) - 1  # odd, every limb of N at its maximum
    top = (1 << (LB * L)) - 1
    for a, b in (((top, top), (top, top)), ((2 * N - 1, 2 * N - 1), (top, top))):
        run_quad(N, [a], [b])
        run_quad(N, [a])
        run_quad(N, [a], lazy_in=True)


def test_quad_operand_shapes_and_lazy_limbs():
    """(h, 0) with h < R, (1, pt) with pt < 2^1036, and lazy input limbs: exact."""
    rng = random.Random(9)
    for bits in (24, 1024):
        N = _rand_n(rng, bits)
        M = N * N
        rinv = pow(R, -1, M)
        h = rng.getrandbits(LB * L)
        r2 = (R * R) % M
        (t, s), = run_quad(N, [(r2 % N, r2 // N)], [(h, 0)])[0]
        assert (t + s * N) % M == h * R % M and t < 3 * N + 1 and s < 3 * N + 1
        pt = rng.getrandbits(1036)
        x = (rng.randrange(2 * N), rng.randrange(2 * N))
        (t, s), = run_quad(N, [x], [(1, pt)])[0]
        assert (t + s * N) % M == (x[0] + x[1] * N) * (1 + N * pt) * rinv % M
        (t, s), = run_quad(N, [x], lazy_in=True)[0]
        X = (x[0] + x[1] * N) % M
        assert (t + s * N) % M == X * X * rinv % M


def test_quad_chain_power():
    """A short square-and-multiply chain through the simulated quad engine (results fed back
    as the next operands, lazy limbs and all): h^e mod N^2."""
    from fedbiomed_amd import workload as W

    N = W.BIPRIME0
    M = N * N
    rng = random.Random(11)
    h, e = rng.getrandbits(256), rng.getrandbits(10) | (1 << 9)
    u = (R * R) % M
    (x,), _, _ = run_quad(N, [(u % N, u // N)], [(h, 0)])
    hr = x
    for bit in bin(e)[3:]:
        (x,), _, _ = run_quad(N, [x])
        if bit == "1":
            (x,), _, _ = run_quad(N, [x], [hr])
    (t, s), = run_quad(N, [x], [(1, 0)])[0]  # * 1 (drops R)
    assert (t + s * N) % M == pow(h, e, M)


def test_quad_dpp_wait_states():
    """Every DPP read of a VGPR is at least 2 wait states after the VALU write of it."""
    for prog in (QMM, QSQ):
        for i, ln in enumerate(prog):
            if "quad_perm" not in ln:
                continue
            src = ln.split(",")[1].split()[0]
            dist = 0
            for prev in reversed(prog[:i]):
                if prev.endswith(":"):
                    break
                if prev.startswith("s_nop"):
                    dist += int(prev.split()[1]) + 1
                    continue
                if prev.startswith("v_") and src in Q.Emitter.dests(prev):
                    break
                dist += 1
                if dist >= 2:
                    break
            assert dist >= 2, (i, ln)
