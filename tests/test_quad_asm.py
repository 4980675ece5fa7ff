"""The generated QUAD and TRIPLE N-adic assembly products (fedbiomed_amd/csrc/fbm_quad_asm.hpp /
fbm_tri_asm.hpp, from tools/gen_quad_asm.py: four / three lanes per ciphertext, 29-bit limbs;
DPP quad_perm exchanges / ds_bpermute broadcasts and DPP wave shifts), run in lockstep for
whole groups (the triple with a trailing all-zero dummy lane, as lane 63 of a wave) on the CPU (tests/asm_sim.py Wave) against Python integers:
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
LB, L = Q.LB, Q.L
MASK = (1 << LB) - 1
R = 1 << (LB * L)
GEOS = {"quad": Q.QUAD, "triple": Q.TRI}
PROGS = {k: (Q.product(False, g), Q.product(True, g)) for k, g in GEOS.items()}
LOOPED_SQ = {k: Q.product(True, g, cyc=False) for k, g in GEOS.items()}  # the table path's square


def limbs(x, n=L):
    return [(x >> (LB * k)) & MASK for k in range(n)]


def qconsts(N):
    """The quad constants the library builds on the host: K'_i = 2^29 - 1 + K_i with
    K = (1 - R) mod N (words 0..35 of the block), np = -N^-1 mod 2^29."""
    K = (1 - R) % N
    return [MASK + v for v in limbs(K)], (-pow(N, -1, 1 << LB)) % (1 << LB)


def run_quad(N, As, Bs=None, lazy_in=False, geo="quad", in_bounds=True, looped=False):
    """As / Bs: lists (one per ciphertext = lane group) of digit pairs; Bs None = square.
    Returns per ciphertext the result digit integers (t, s), the max limb and the counts.
    geo "triple": groups of 3 lanes and a trailing dummy lane (zero column, e0 = 0, N = 0,
    permute source itself), as lane 63 of a triple-engine wave.  in_bounds: the operands are
    within the engine's documented bounds, so the top lane hands nothing up (checked: the
    dummy column stays zero)."""
    g = GEOS[geo]
    G, ML, ROWB, D1 = g.G, g.M, g.ROWB, g.D1
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
        for l in range(G):
            tid = G * c + l
            if Bs is not None:
                bl, bh = limbs(Bs[c][0]), limbs(Bs[c][1])
                for r in range(ML):
                    glb[BB + tid * 4 + r * 1024] = bl[ML * l + r]
                    glb[BB + tid * 4 + (ML + r) * 1024] = bh[ML * l + r]
            args = {"ac": ac, "al": ac + ML * l * ROWB, "b": tid * 4, "bb": BB, "QK": QK, "np": np_,
                    "e0": 1 if l == 0 else 0, "bp": 4 * G * c,
                    "mq": MASK if l == 0 else 0}
            for r in range(ML):
                args[f"n{r}"] = nl[ML * l + r]
            lanes.append(Lane(args, lds=lds, glb=glb, smem=smem))
    if G == 3:  # the wave's dummy lane: its own all-zero column, contributes nothing
        tid, ac = G * len(As), 4 * len(As)
        if Bs is not None:
            for j in range(2 * ML):
                glb[BB + tid * 4 + j * 1024] = 0
        args = {"ac": ac, "al": ac, "b": tid * 4, "bb": BB, "QK": QK, "np": np_, "e0": 0, "bp": 4 * tid, "mq": 0}
        args.update({f"n{r}": 0 for r in range(ML)})
        lanes.append(Lane(args, lds=lds, glb=glb, smem=smem))
    mm, sq = PROGS[geo]
    if looped:
        sq = LOOPED_SQ[geo]
    counts = Wave(lanes).run(mm if Bs is not None else sq)
    if G == 3 and in_bounds:
        assert all(lds.get(4 * len(As) + k * ROWB, 0) == 0 for k in range(2 * L)), "dummy column disturbed"
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


@pytest.mark.parametrize("geo", ["quad", "triple"])
@pytest.mark.parametrize("bits", [2, 24, 1024])
def test_quad_product_and_square(bits, geo):
    rng = random.Random(100 + bits)
    N = _rand_n(rng, bits)
    M = N * N
    rinv = pow(R, -1, M)
    As = [(2 * N - 1, 2 * N - 1)] + [(rng.randrange(2 * N), rng.randrange(2 * N)) for _ in range(2)]
    Bs = [(2 * N - 1, 2 * N - 1)] + [(rng.randrange(2 * N), rng.randrange(2 * N)) for _ in range(2)]
    got, top, counts = run_quad(N, As, Bs, geo=geo)
    assert top < (1 << LB) + (1 << 11)
    assert counts["v_mad_u64_u32"] == Q.product_mads(False, GEOS[geo])
    for a, b, (t, s) in zip(As, Bs, got):
        A, B = (a[0] + a[1] * N) % M, (b[0] + b[1] * N) % M
        assert (t + s * N) % M == A * B * rinv % M
        assert t < 2 * N and s < 2 * N
    got, top, counts = run_quad(N, As, geo=geo)
    assert counts["v_mad_u64_u32"] == Q.product_mads(True, GEOS[geo])
    for a, (t, s) in zip(As, got):
        A = (a[0] + a[1] * N) % M
        assert (t + s * N) % M == A * A * rinv % M
        assert t < 2 * N and s < 2 * N


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_quad_worst_case_columns(geo):
    """All-ones limbs (every operand limb 2^29 - 1, and lazy ones above it): the largest column
    sums the bound allows; the simulator's overflow asserts are the check."""
    N = (1 << 1024) - 1  # odd, every limb of N at its maximum
    top = (1 << (LB * L)) - 1
    for a, b in (((top, top), (top, top)), ((2 * N - 1, 2 * N - 1), (top, top))):
        run_quad(N, [a], [b], geo=geo, in_bounds=False)
        run_quad(N, [a], geo=geo, in_bounds=False)
        run_quad(N, [a], lazy_in=True, geo=geo, in_bounds=False)


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_quad_operand_shapes_and_lazy_limbs(geo):
    """(h, 0) with h < R, (1, pt) with pt < 2^1036, and lazy input limbs: exact."""
    rng = random.Random(9)
    for bits in (24, 1024):
        N = _rand_n(rng, bits)
        M = N * N
        rinv = pow(R, -1, M)
        h = rng.getrandbits(LB * L)
        r2 = (R * R) % M
        (t, s), = run_quad(N, [(r2 % N, r2 // N)], [(h, 0)], geo=geo)[0]
        assert (t + s * N) % M == h * R % M and t < 3 * N + 1 and s < 3 * N + 1
        pt = rng.getrandbits(1036)
        x = (rng.randrange(2 * N), rng.randrange(2 * N))
        (t, s), = run_quad(N, [x], [(1, pt)], geo=geo)[0]
        assert (t + s * N) % M == (x[0] + x[1] * N) * (1 + N * pt) * rinv % M
        (t, s), = run_quad(N, [x], lazy_in=True, geo=geo)[0]
        X = (x[0] + x[1] * N) % M
        assert (t + s * N) % M == X * X * rinv % M


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_quad_chain_power(geo):
    """A short square-and-multiply chain through the simulated quad engine (results fed back
    as the next operands, lazy limbs and all): h^e mod N^2."""
    from fedbiomed_amd import workload as W

    N = W.BIPRIME0
    M = N * N
    rng = random.Random(11)
    h, e = rng.getrandbits(256), rng.getrandbits(10) | (1 << 9)
    u = (R * R) % M
    (x,), _, _ = run_quad(N, [(u % N, u // N)], [(h, 0)], geo=geo)
    hr = x
    for bit in bin(e)[3:]:
        (x,), _, _ = run_quad(N, [x], geo=geo)
        if bit == "1":
            (x,), _, _ = run_quad(N, [x], [hr], geo=geo)
    (t, s), = run_quad(N, [x], [(1, 0)], geo=geo)[0]  # * 1 (drops R)
    assert (t + s * N) % M == pow(h, e, M)


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_quad_dpp_wait_states(geo):
    """Every DPP read of a VGPR is at least 2 wait states after the VALU write of it."""
    for prog in PROGS[geo]:
        for i, ln in enumerate(prog):
            if not Q.is_dpp(ln):
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


def _lds_waits_ok(prog, g):
    """Every read of a ds_bpermute / ds_read destination comes after an s_waitcnt that has
    retired that LDS op (LDS ops return in order; lgkmcnt(k) = at most k still in flight).
    Loop back-edges are followed once (the row pairs are the steady state)."""
    lab = {ln[:-1]: i for i, ln in enumerate(prog) if ln.endswith(":")}
    pending = []  # destinations of in-flight LDS ops, oldest first

    def reads(ln):
        op, _, rest = ln.partition(" ")
        toks = [t.strip().split()[0] for t in rest.split(",")[1:]] if rest else []
        if op.startswith("ds_write"):
            toks = [t.strip().split()[0] for t in rest.split(",")]
        return {t for t in toks if t.startswith("v") and not t.startswith("v[")} | \
            {f"v{k}" for t in toks if t.startswith("v[") for k in range(int(t[2:-1].split(":")[0]),
                                                                       int(t[2:-1].split(":")[1]) + 1)}

    seen_back = set()
    i = 0
    while i < len(prog):
        ln = prog[i]
        op = ln.split(" ")[0]
        if op == "s_waitcnt" and "lgkmcnt" in ln:
            k = int(ln.split("lgkmcnt(")[1].split(")")[0])
            pending = pending[len(pending) - k:] if k else []
        else:
            r = reads(ln)
            for d in pending:
                assert not (d & r if isinstance(d, frozenset) else d in r), \
                    f"read of {d} before its LDS op retired: {i}: {ln}"
            if op in ("ds_read_b32", "ds_read_b64", "ds_bpermute_b32"):
                d = ln.split(" ")[1].rstrip(",")
                if d.startswith("v["):  # a pair: both registers pending (one LDS op)
                    lo, hi = (int(x) for x in d[2:-1].split(":"))
                    d = frozenset(f"v{k}" for k in range(lo, hi + 1))
                pending.append(d)
        if op == "s_cbranch_scc1" and i not in seen_back:
            seen_back.add(i)
            i = lab[ln.split(" ")[1].rstrip("bf")]
            continue
        i += 1
    return True


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_lds_results_waited_for(geo):
    for prog in PROGS[geo]:
        assert _lds_waits_ok(prog, GEOS[geo])


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_cyclic_band_square_covers_each_product_once(geo):
    """The cyclic-band triangular square (gen_quad_asm.cyc_active): over the 36 rows and the G lanes,
    x_a * x_b (a < b) is added with total weight 2 and x_a^2 with weight 1 -- each pair once doubled or
    twice undoubled -- and the rows' instruction streams are the same in every lane (activity depends
    on (r - i) mod M only)."""
    g = GEOS[geo]
    weight = {}
    for i in range(L):
        for r, dbl in Q.cyc_active(g, i):
            for lane in range(g.G):
                j = g.M * lane + r
                key = (min(i, j), max(i, j))
                weight[key] = weight.get(key, 0) + (2 if dbl else 1)
    for a in range(L):
        for b in range(a, L):
            assert weight.get((a, b), 0) == (1 if a == b else 2), (a, b, weight.get((a, b)))
    per_row = [len(Q.cyc_active(g, i)) for i in range(L)]
    assert per_row == [g.M // 2 + 1] * L  # 7 of 12 (triple), 5 of 9 (quad)


SHORT = {k: Q.mul_short(g) for k, g in GEOS.items()}


def run_short_group(N, As, hs, geo):
    """The group engines' short-base product A h 2^-261 (mod N^2) for whole groups: h's 9 limbs in
    LDS rows HROW.. of each ciphertext's column, the pairs (D_j, 0) (D = N - 2^261, then 12 zero
    pairs for the triple's dummy lane) in LDS.  Returns per ciphertext (t, s), the max limb, counts."""
    g = GEOS[geo]
    G, ML, ROWB = g.G, g.M, g.ROWB
    _, np_ = qconsts(N)
    DADDR = 0x40000
    lds = {}
    for j, v in enumerate(limbs(N - (1 << (LB * Q.KS))) + [0] * 12):
        lds[DADDR + 8 * j] = v
        lds[DADDR + 8 * j + 4] = 0
    nl = limbs(N)
    lanes = []
    for c in range(len(As)):
        ac = 4 * c
        for k, v in enumerate(limbs(As[c][0]) + limbs(As[c][1])):
            lds[ac + k * ROWB] = v
        for k, v in enumerate(limbs(hs[c], Q.KS + 1)):  # + the prefetch row (0)
            lds[ac + (Q.HROW + k) * ROWB] = v
        for l in range(G):
            args = {"ac": ac, "al": ac + ML * l * ROWB, "dl": DADDR + 8 * ML * l, "np": np_,
                    "e0": 1 if l == 0 else 0, "bp": 4 * G * c,
                    "mq": MASK if l == 0 else 0}
            args.update({f"n{r}": nl[ML * l + r] for r in range(ML)})
            lanes.append(Lane(args, lds=lds))
    if G == 3:
        tid, ac = G * len(As), 4 * len(As)
        args = {"ac": ac, "al": ac, "dl": DADDR + 8 * L, "np": np_, "e0": 0, "bp": 4 * tid, "mq": 0}
        args.update({f"n{r}": 0 for r in range(ML)})
        lanes.append(Lane(args, lds=lds))
    counts = Wave(lanes).run(SHORT[geo])
    if G == 3:
        assert all(lds.get(4 * len(As) + k * ROWB, 0) == 0 for k in range(2 * L)), "dummy column disturbed"
    out, top = [], 0
    for c in range(len(As)):
        col = [lds[4 * c + k * ROWB] for k in range(2 * L)]
        top = max(top, max(col))
        out.append((sum(v << (LB * k) for k, v in enumerate(col[:L])), sum(v << (LB * k) for k, v in enumerate(col[L:]))))
    return out, top, counts


@pytest.mark.parametrize("geo", ["quad", "triple"])
@pytest.mark.parametrize("bits", [263, 1024])
def test_group_short_product(bits, geo):
    """x h 2^-261 (mod N^2) for h < 2^261 and digits < 2N (the worst case included) over whole
    groups: digits < 3N + 2, lazy limbs in bound, 9 rows of 4 M + 1 multiplies per lane."""
    rng = random.Random(300 + bits)
    N = _rand_n(rng, bits)
    M = N * N
    f = pow(2, -LB * Q.KS, M)
    As = [(2 * N - 1, 2 * N - 1)] + [(rng.randrange(2 * N), rng.randrange(2 * N)) for _ in range(2)]
    hs = [(1 << (LB * Q.KS)) - 1, rng.getrandbits(256), rng.getrandbits(LB * Q.KS)]
    got, top, counts = run_short_group(N, As, hs, geo)
    assert top < (1 << LB) + (1 << 11)
    assert counts["v_mad_u64_u32"] == Q.ms_mads(GEOS[geo]) == Q.KS * (4 * GEOS[geo].M + 1)
    for a, h, (t, s) in zip(As, hs, got):
        A = (a[0] + a[1] * N) % M
        assert (t + s * N) % M == A * h * f % M
        assert t < 3 * N and s < 3 * N + 2


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_group_short_chain_power(geo):
    """The short path's chain through the simulated group engine: (h, 0) raw, a squaring per
    exponent bit and a short product per 1 bit, then the host constant C (one general product):
    h^e R, and * 1 -> h^e."""
    from fedbiomed_amd import workload as W

    N = W.BIPRIME0
    M = N * N
    rng = random.Random(13)
    h, e = rng.getrandbits(256), rng.getrandbits(10) | (1 << 9)
    s = e.bit_length() - 1
    x = (h, 0)
    for bit in bin(e)[3:]:
        (x,), _, _ = run_quad(N, [x], geo=geo)
        if bit == "1":
            (x,), _, _ = run_short_group(N, [x], [h], geo)
    C = pow(2, LB * L * ((1 << s) + 1) + LB * Q.KS * (e - (1 << s)), M)
    (x,), _, _ = run_quad(N, [(C % N, C // N)], [x], geo=geo)
    (t, s_), = run_quad(N, [x], [(1, 0)], geo=geo)[0]
    assert (t + s_ * N) % M == pow(h, e, M)


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_group_short_product_waits(geo):
    """DPP wait states and LDS results waited for in the short product too."""
    prog = SHORT[geo]
    assert _lds_waits_ok(prog, GEOS[geo])
    for i, ln in enumerate(prog):
        if Q.is_dpp(ln):
            src = ln.split(",")[1].split()[0]
            dist = 0
            for prev in reversed(prog[:i]):
                if prev.startswith("s_nop"):
                    dist += int(prev.split()[1]) + 1
                    continue
                if prev.startswith("v_") and src in Q.Emitter.dests(prev):
                    break
                dist += 1
                if dist >= 2:
                    break
            assert dist >= 2, (i, ln)


@pytest.mark.parametrize("geo", ["quad", "triple"])
def test_looped_square_equals_cyclic_band_square(geo):
    """The table path's looped square (the rows as a runtime loop, no triangular skip) gives the
    cyclic-band square's residues bit for bit (same column totals at every quotient)."""
    rng = random.Random(77)
    from fedbiomed_amd import workload as W

    N = W.BIPRIME0
    As = [(2 * N - 1, 2 * N - 1)] + [(rng.randrange(2 * N), rng.randrange(2 * N)) for _ in range(2)]
    got, _, _ = run_quad(N, As, geo=geo)
    got2, _, _ = run_quad(N, As, geo=geo, looped=True)
    assert got == got2


def test_group_column_bounds_proved_without_mid_reduce():
    """Round 4 dropped the group engines' mid-product reduction: a column lives in a lane's window for
    at most M rows (a retire hands only its low 29 bits to the lane below), so it restarts below
    2^29 + 2^10 whenever it changes lanes.  tests/asm_bounds.py runs every group program (the cyclic-band
    square, the looped square, the general product, the short-base product) on intervals -- one abstract
    lane holding the hull over the group's lanes, every operand limb in [0, 2^29 + 2^10) (the lazy limbs),
    any N limbs, np, K' -- and no 64-bit multiply-add can overflow."""
    from tests.asm_bounds import BoundLane

    for g in (Q.QUAD, Q.TRI):
        for prog in (Q.square_cyc(g), Q.product(False, g), Q.product(True, g, cyc=False), Q.mul_short(g)):
            assert not any(ln.startswith("v_mad_u64_u32") and ", 8," in ln for ln in prog)  # no mid-reduce left
            QK, BB, DL = 0x4000, 0x100000, 0x40000
            lim = (0, MASK + (1 << 10))
            lds = {k * g.ROWB: lim for k in range(2 * L + 20)}
            lds.update({DL + 4 * j: ((0, MASK) if j % 2 == 0 else (0, 0)) for j in range(2 * g.M + 2)})
            args = {"ac": 0, "al": 0, "QK": QK, "np": (0, MASK), "e0": (0, 1), "mq": (0, MASK), "bp": 0, "b": 0, "bb": BB,
                    "dl": DL}
            args.update({f"n{r}": (0, MASK) for r in range(g.M)})
            lane = BoundLane(args, lds=lds, smem={QK + 4 * i: (MASK, 2 * MASK) for i in range(40)},
                             glb={BB + j * 1024: lim for j in range(2 * g.M)})
            lane.run(prog)
            assert lane.max_mad < 0.6 * 2**64
