"""The generated N-adic assembly product (fedbiomed_amd/csrc/fbm_nadic_asm.hpp, from
tools/gen_nadic_asm.py), run instruction by instruction for one lane on the CPU
(tests/asm_sim.py), against Python integers: X*Y*R^-1 mod N^2 for digits < 2N (and the
one-off operand shapes the exponentiation uses), digits staying < 2N."""

import importlib.util
import os
import random

import pytest

from tests.asm_sim import Lane  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LB, L = 29, 36
MASK = (1 << LB) - 1
R = 1 << (LB * L)


def _gen():
    spec = importlib.util.spec_from_file_location("gen_nadic_asm", os.path.join(ROOT, "tools", "gen_nadic_asm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


GEN = _gen()
MM, SQ, SQ_PLAIN = GEN.product(False), GEN.square_tri(), GEN.product(True)
SQ_UNROLLED = GEN.square_unrolled()


def limbs(x, n=L):
    return [(x >> (LB * k)) & MASK for k in range(n)]


def consts(N):
    """80-word constants block: N_0..N_9 at words 0..9, N_10..N_35 at 16..41, K'_0..K'_35 at
    42..77 (the layout fbm_capi.hip's host setup writes)."""
    K = (1 - R) % N
    kp = [MASK + v for v in limbs(K)]
    nl = limbs(N)
    words = [0] * 80
    words[0:10] = nl[0:10]
    words[16:16 + 26] = nl[10:36]
    words[42:78] = kp
    np_ = (-pow(N, -1, 1 << LB)) % (1 << LB)
    return words, np_


def sq_pairs(N):
    """The unrolled square's initial s window (round 4, K' folded): 2^29 - 1 + P'_j, P' = (K - E) mod N
    (the library's QuadCtx::sqp, written to the constants block and copied to LDS by the kernel)."""
    K = (1 - R) % N
    return [MASK + v for v in limbs((K - GEN.sq_kfold_extra()) % N)]


KADDR = 76 * 1024  # the pairs' LDS address in these runs (outside the column's 72 + 1 rows)


def run(N, a, b=None, square=None):
    """a, b: (digit0, digit1) pairs; b None = square (`square`: which square body).
    Returns the result digits and the executed-instruction counts."""
    words, np_ = consts(N)
    NK, BB = 0x4000, 0x100000
    smem = {NK + 4 * i: w for i, w in enumerate(words)}
    lds = {}
    for k, v in enumerate(limbs(a[0]) + limbs(a[1])):
        lds[k * 1024] = v
    for j, v in enumerate(sq_pairs(N)):
        lds[KADDR + 8 * j] = v
        lds[KADDR + 8 * j + 4] = 0
    glb = {}
    if b is not None:
        for k, v in enumerate(limbs(b[0]) + limbs(b[1])):
            glb[BB + k * 1024] = v
    lane = Lane({"a": 0, "b": 0, "bb": BB, "k": KADDR, "NK": NK, "np": np_}, lds=lds, glb=glb, smem=smem)
    counts = lane.run(MM if b is not None else (square or SQ))
    out = [lds[k * 1024] for k in range(2 * L)]
    assert all(v <= MASK for v in out)
    d0 = sum(v << (LB * k) for k, v in enumerate(out[:L]))
    d1 = sum(v << (LB * k) for k, v in enumerate(out[L:]))
    return d0, d1, counts


def _rand_n(rng, bits):
    return rng.getrandbits(bits) | (1 << (bits - 1)) | 1


MS = GEN.mul_short_reg()
KS = GEN.KS


def run_short(N, a, h):
    """The short-base product a * h * 2^-(29 KS) (mod N^2): a = (digit0, digit1) in the LDS column,
    h < 2^(29 KS) in registers (%[h0] .. %[h8]), the pairs (D'_j, 0) in LDS, D'_j = D_j + (2^29 - 1)
    [j < KS] + [j == 0], D = N - 2^(29 KS) (the kernel builds them from the constants block)."""
    words, np_ = consts(N)
    NK, DADDR = 0x4000, 74 * 1024
    smem = {NK + 4 * i: w for i, w in enumerate(words)}
    lds = {}
    for k, v in enumerate(limbs(a[0]) + limbs(a[1])):
        lds[k * 1024] = v
    for j, v in enumerate(limbs(N - (1 << (LB * KS)))):
        lds[DADDR + 8 * j] = v + (MASK if j < KS else 0) + (1 if j == 0 else 0)
        lds[DADDR + 8 * j + 4] = 0
    args = {"a": 0, "d": DADDR, "NK": NK, "np": np_}
    args.update({f"h{i}": v for i, v in enumerate(limbs(h, KS))})
    lane = Lane(args, lds=lds, smem=smem)
    counts = lane.run(MS)
    out = [lds[k * 1024] for k in range(2 * L)]
    assert all(v <= MASK for v in out)
    d0 = sum(v << (LB * k) for k, v in enumerate(out[:L]))
    d1 = sum(v << (LB * k) for k, v in enumerate(out[L:]))
    return d0, d1, counts


@pytest.mark.parametrize("bits", [263, 700, 1024])
def test_nadic_asm_short_product(bits):
    """X h 2^-261 (mod N^2) for h < 2^261 (one FDH digest) and digits < 2N (a square's output,
    the worst case included): digits < 3N + 2, 1 305 multiplies, every column below 2^64."""
    rng = random.Random(bits)
    N = _rand_n(rng, bits)
    M = N * N
    f = pow(2, -LB * KS, M)
    for trial in range(4):
        a = (rng.randrange(2 * N), rng.randrange(2 * N))
        h = rng.getrandbits(LB * KS)
        if trial == 0:
            a, h = (2 * N - 1, 2 * N - 1), (1 << (LB * KS)) - 1
        if trial == 1:
            h = rng.getrandbits(256)
        A = (a[0] + a[1] * N) % M
        t, s, counts = run_short(N, a, h)
        assert (t + s * N) % M == A * h * f % M
        assert t < 3 * N and s < 3 * N + 2
        assert counts["v_mad_u64_u32"] + counts.get("v_mad_i64_i32", 0) == GEN.ms_mads() == 1305
        # the next squaring brings the digits back below 2N
        t2, s2, _ = run(N, (t, s))
        assert (t2 + s2 * N) % M == A * A * h * h * f * f * pow(R, -1, M) % M
        assert t2 < 2 * N and s2 < 2 * N


def test_nadic_asm_binary_chain_with_short_products():
    """h^e mod N^2 the way jl_exp_kernel's short path sequences it: (h, 0) raw, then per exponent
    bit below the top a squaring and, on a 1, a short product; one general product with the
    host-built constant C = 2^(1044 (2^s + 1) + 261 (e - 2^s)) mod N^2 (s = bit length of e - 1)
    brings the chain to h^e R, the Montgomery form the epilogue expects."""
    from fedbiomed_amd import workload as W

    N = W.BIPRIME0
    M = N * N
    rng = random.Random(11)
    h, e = rng.getrandbits(256), rng.getrandbits(24) | (1 << 23)
    s = e.bit_length() - 1
    x = (h, 0)
    for bit in bin(e)[3:]:
        x = run(N, x, square=SQ_UNROLLED)[:2]  # the shipped square
        if bit == "1":
            x = run_short(N, x, h)[:2]
    E = LB * L * ((1 << s) + 1) + LB * KS * (e - (1 << s))
    C = pow(2, E, M)
    y = run(N, (C % N, C // N), x)[:2]
    assert (y[0] + y[1] * N) % M == pow(h, e, M) * R % M


MM_NUDE = GEN.product(False, nude=True)


@pytest.mark.parametrize("bits", [2, 263, 1024])
def test_nadic_asm_nude_product(bits):
    """fbm_na_mm_nude (round 4): the encrypt's last product by nude = N pt + 1 = (1, pt) with only pt's 36
    rows in global memory (digit 0 as immediates) -- the general product's result bit for bit, pt up to
    the one-off operand bound 2^1036 (a negative packing's M - |pt|) included."""
    rng = random.Random(900 + bits)
    N = _rand_n(rng, bits)
    words, np_ = consts(N)
    NK, BB = 0x4000, 0x100000
    for trial in range(3):
        a = (rng.randrange(2 * N), rng.randrange(2 * N))
        pt = [rng.getrandbits(1024), (1 << 1036) - 1, 0][trial]
        t, s, _ = run(N, a, (1, pt))
        lds = {k * 1024: v for k, v in enumerate(limbs(a[0]) + limbs(a[1]))}
        glb = {BB + k * 1024: v for k, v in enumerate(limbs(pt))}
        lane = Lane({"a": 0, "b": 0, "bb": BB, "NK": NK, "np": np_}, lds=lds, glb=glb,
                    smem={NK + 4 * i: w for i, w in enumerate(words)})
        lane.run(MM_NUDE)
        out = [lds[k * 1024] for k in range(2 * L)]
        d0 = sum(v << (LB * k) for k, v in enumerate(out[:L]))
        d1 = sum(v << (LB * k) for k, v in enumerate(out[L:]))
        assert (d0, d1) == (t, s), trial
    assert sum(1 for ln in MM_NUDE if ln.startswith("global_load_dword")) == L  # digit 1's rows only


@pytest.mark.parametrize("bits", [2, 24, 1024])
def test_nadic_asm_product_and_square(bits):
    rng = random.Random(bits)
    N = _rand_n(rng, bits)  # bits = 2: N = 3, a divisor of R - 1 (K = 0, K'_i = 2^29 - 1)
    M = N * N
    rinv = pow(R, -1, M)
    for trial in range(3):
        a = (rng.randrange(2 * N), rng.randrange(2 * N))
        b = (rng.randrange(2 * N), rng.randrange(2 * N))
        if trial == 0:
            a, b = (2 * N - 1, 2 * N - 1), (2 * N - 1, 2 * N - 1)
        A, B = (a[0] + a[1] * N) % M, (b[0] + b[1] * N) % M
        t, s, counts = run(N, a, b)
        assert (t + s * N) % M == A * B * rinv % M
        assert t < 2 * N and s < 2 * N
        assert counts["v_mad_u64_u32"] == GEN.mm_mads() == 36 * 181 + 68
        t, s, counts = run(N, a)
        assert (t + s * N) % M == A * A * rinv % M
        assert t < 2 * N and s < 2 * N
        assert counts["v_mad_u64_u32"] == 4658
        # the triangular square is the plain square bit for bit (same column totals at
        # every quotient -- the mid-product reduction moves value up a column, never out of
        # one before its quotient -- so the same quotients and the same result)
        t2, s2, c2 = run(N, a, square=SQ_PLAIN)
        assert (t2, s2) == (t, s) and c2["v_mad_u64_u32"] == 36 * 145 + 68
        # the unrolled square (the shipped one: K' folded, the mid-product reduction on 34 slots):
        # the same t digit (the same quotients), an s digit equal mod N (its constant is P' + E, not
        # K), no jumps or m0
        t3, s3, c3 = run(N, a, square=SQ_UNROLLED)
        # (its constant adds up to (R + E) / R < 10 to s: below 2N needs N > 2^262 -- the short path's
        # domain, the only one that runs this square; smaller N take the looped square)
        assert t3 == t and (s3 - s) % N == 0 and (s3 < 2 * N or N < (1 << 262))
        assert c3["v_mad_u64_u32"] + c3["v_mad_i64_i32"] == GEN.sq_mads() == 4624
        assert "s_setpc_b64" not in c3 and "s_movrels_b32" not in c3 and "v_sub_u32" not in c3


def test_nadic_asm_wide_operands():
    """(h, 0) with h < R (the FDH digest entering the exponentiation) and (1, pt) with
    pt < 2^1024 (N*pt + 1): results stay exact, digits < 3N + 1."""
    rng = random.Random(5)
    for bits in (24, 1024):
        N = _rand_n(rng, bits)
        M = N * N
        rinv = pow(R, -1, M)
        h = rng.getrandbits(LB * L)
        r2 = (R * R) % M
        a = (r2 % N, r2 // N)
        t, s, _ = run(N, a, (h, 0))
        assert (t + s * N) % M == h * R % M
        assert t < 3 * N + 1 and s < 3 * N + 1
        pt = rng.getrandbits(1024)
        x = (rng.randrange(2 * N), rng.randrange(2 * N))
        t, s, _ = run(N, x, (1, pt))
        assert (t + s * N) % M == (x[0] + x[1] * N) * (1 + N * pt) * rinv % M


def test_library_constants_match_and_drive_the_asm():
    """The constants the library builds on the host (fbm_test_nadic_consts: N limbs, K'_i,
    R^2 / R^3 digits, np) equal the formulas above, and a short square-and-multiply chain of the
    simulated assembly on them gives h^e mod N^2 for the default biprime."""
    import numpy as np

    from fedbiomed_amd import _build, _native, workload as W

    _build.build()
    lib = _native.load_test()
    for N in (W.BIPRIME0, 0xC9F2B5, (1 << 1023) + 12345677, 3, 5):  # 3, 5 divide R - 1: K = 0
        n32 = np.frombuffer(N.to_bytes(128, "little"), dtype=np.uint32).copy()
        nk = np.zeros(80, np.uint32)
        r2 = np.zeros(2 * L, np.uint32)
        r3 = np.zeros(2 * L, np.uint32)
        npv = np.zeros(1, np.uint32)
        assert lib.fbm_test_nadic_consts(n32.ctypes.data, nk.ctypes.data, r2.ctypes.data, r3.ctypes.data,
                                         npv.ctypes.data) == 0
        words, np_ = consts(N)
        assert [int(v) for v in nk] == words
        assert int(npv[0]) == np_
        for e, got in ((2, r2), (3, r3)):
            u = pow(R, e, N * N)
            assert [int(v) for v in got] == limbs(u % N) + limbs(u // N)
    # h^e mod N^2 through the simulated engine, as jl_exp_kernel sequences it (binary method)
    N = W.BIPRIME0
    M = N * N
    rng = random.Random(9)
    h, e = rng.getrandbits(256), rng.getrandbits(12) | (1 << 11)
    u = (R * R) % M
    x = run(N, (u % N, u // N), (h, 0))[:2]          # h R
    hr = x
    for bit in bin(e)[3:]:
        x = run(N, x)[:2]
        if bit == "1":
            x = run(N, x, hr)[:2]
    # a wide h (FDH retries on a small modulus): h R = h_lo R + h_hi R^2, summed digit-wise
    Ns = 0xC9F2B5
    Ms = Ns * Ns
    hw = rng.getrandbits(1792)
    hl, hh = hw % R, hw // R
    u2, u3 = pow(R, 2, Ms), pow(R, 3, Ms)
    lo = run(Ns, (u2 % Ns, u2 // Ns), (hl, 0))[:2]
    hi = run(Ns, (u3 % Ns, u3 // Ns), (hh, 0))[:2]
    s0, s1 = lo[0] + hi[0], lo[1] + hi[1]
    assert (s0 + s1 * Ns) % Ms == hw * R % Ms and s0 < 6 * Ns + 2 and s1 < 6 * Ns + 2
    sq = run(Ns, (s0, s1))[:2]
    assert (sq[0] + sq[1] * Ns) % Ms == hw * hw * R % Ms
    pt = rng.getrandbits(1000)
    t, s, _ = run(N, x, (1, pt))                       # * (N pt + 1), drops R
    assert (t + s * N) % M == (1 + N * pt) * pow(h, e, M) % M
    assert t <= N and s < 2 * N


def test_library_short_path_constants():
    """The short path's per-call words as the library builds them (fbm_test_short_consts): |key|'s
    words, the digits of C = 2^(1044 (2^s + 1) + 261 (|key| - 2^s)) mod N^2, D = N - 2^261 -- against
    Python integers, for the default biprime and random odd moduli, 2 040-bit and short keys; moduli
    at or below 2^262 (and even ones) are outside the path (-2), a zero key has no chain (-1)."""
    import numpy as np

    from fedbiomed_amd import _build, _native, workload as W

    _build.build()
    lib = _native.load_test()
    rng = random.Random(21)
    cases = [(W.BIPRIME0, W.jl_user_key(0)), (W.BIPRIME0, 1), (W.BIPRIME0, 3), (_rand_n(rng, 1024), rng.getrandbits(2040)),
             (_rand_n(rng, 600), rng.getrandbits(900) | 1), ((1 << 262) + 1, 12345), (W.BIPRIME0, 0),
             ((1 << 262) - 1, 7), (W.BIPRIME0 + 1, 7)]
    for N, key in cases:
        n32 = np.frombuffer(N.to_bytes(128, "little"), dtype=np.uint32).copy()
        k64 = np.frombuffer(abs(key).to_bytes(256, "little"), dtype=np.uint32).copy()
        kw, corr, d = np.zeros(64, np.uint32), np.zeros(72, np.uint32), np.zeros(36, np.uint32)
        r = lib.fbm_test_short_consts(n32.ctypes.data, k64.ctypes.data, kw.ctypes.data, corr.ctypes.data, d.ctypes.data)
        if N <= (1 << 262) or N % 2 == 0:
            assert r == -2
            continue
        assert [int(v) for v in d] == limbs(N - (1 << (LB * KS)))
        e = abs(key)
        if e == 0:
            assert r == -1
            continue
        s = e.bit_length() - 1
        assert r == s and [int(v) for v in kw] == list(k64)
        C = pow(2, LB * L * ((1 << s) + 1) + LB * KS * (e - (1 << s)), N * N)
        assert [int(v) for v in corr] == limbs(C % N) + limbs(C // N)


def _bound_lane(top, pairs_at=None, pair_iv=None):
    """A lane of interval values: the LDS column's limbs 0..34 of each digit in [0, 2^29), limb 35 in
    [0, top]; N's 29-bit limbs in [0, 2^29) (N_35 < 2^9: N < 2^1024), K'_j = 2^29 - 1 + K_j likewise;
    np any 29-bit value; optional (lo, 0) pairs at `pairs_at` (%[k] / %[d]) with lo in pair_iv(j)."""
    from tests.asm_bounds import BoundLane

    NK = 0x4000
    smem = {NK + 4 * w: (0, 0) for w in range(80)}
    for j in range(L):
        w = j if j < 10 else 6 + j
        nmax = MASK if j < L - 1 else (1 << 9) - 1
        smem[NK + 4 * w] = (0, nmax)
        smem[NK + 4 * (42 + j)] = (MASK, MASK + nmax)
    lds = {k * 1024: (0, MASK if k % L < L - 1 else top) for k in range(2 * L)}
    lds[2 * L * 1024] = (0, MASK)
    args = {"a": 0, "NK": NK, "np": (0, MASK)}
    if pairs_at is not None:
        args["k"] = args["d"] = (pairs_at, pairs_at)
        for j in range(L):
            lds[pairs_at + 8 * j] = pair_iv(j)
            lds[pairs_at + 8 * j + 4] = (0, 0)
    return BoundLane(args, lds=lds, smem=smem)


def test_column_bounds_proved_for_every_operand():
    """tests/asm_bounds.py runs the shipped square and short product on intervals: for EVERY input
    within the products' bounds (digits < 2^1026: limb 35 < 2^11; any N < 2^1024; any np; h < 2^261)
    no 64-bit multiply-add overflows and no quotient subtraction goes negative -- the proof behind
    the mid-product reduction's 34 kept slots (of 68) and the folded K' / D' constants -- and a
    reduction dropped from any one kept slot breaks it (the set is minimal)."""
    from tests.asm_bounds import Overflow

    top = (1 << 11) - 1
    nmax = lambda j: MASK if j < L - 1 else (1 << 9) - 1  # noqa: E731
    kp = lambda j: (MASK, MASK + nmax(j))  # noqa: E731  (2^29 - 1 + a limb of a number < N)
    dp = lambda j: (MASK + (j == 0), 2 * MASK + 1) if j < KS else (0, nmax(j))  # noqa: E731  (D'_j)
    _bound_lane(top, KADDR, kp).run(SQ_UNROLLED)
    lane = _bound_lane(top, KADDR, dp)
    lane.args.update({f"h{i}": (0, MASK) for i in range(KS)})
    lane.run(MS)
    # the encrypt's last product by (1, pt), pt < 2^1036 (a negative packing's M - |pt| included)
    lane = _bound_lane(top)
    BB = 0x100000
    lane.args.update({"b": (0, 0), "bb": (BB, BB)})
    lane.glb.update({BB + k * 1024: (0, MASK if k < L - 1 else (1 << 21) - 1) for k in range(L)})
    lane.run(MM_NUDE)
    keep = GEN.SQ_MID_KEEP
    try:
        for part in (0, 1):
            for k in sorted(keep[part]):
                GEN.SQ_MID_KEEP = (keep[0] - {k}, keep[1]) if part == 0 else (keep[0], keep[1] - {k})
                with pytest.raises(Overflow):
                    _bound_lane(top, KADDR, kp).run(GEN.square_unrolled())
    finally:
        GEN.SQ_MID_KEEP = keep
