#!/usr/bin/env python3
"""Generate fedbiomed_amd/csrc/fbm_nadic_asm.hpp: the gfx950 assembly Montgomery product
modulo N^2 in N-adic form (the Joye-Libert exponentiation engine).

Why N-adic: the JL modulus is N^2 with N known (1024-bit biprime).  A residue X mod N^2 is
carried as two 36-limb digits (x0, x1), X = x0 + x1 N (mod N^2), and since N^2 = 0 the
product needs no x1*y1 term:

    X Y = x0 y0 + N (x0 y1 + x1 y0)                      (mod N^2)

With R = 2^1044 (36 limbs of 29 bits) and one Montgomery reduction modulo N of x0 y0,
x0 y0 + m N = t R  (m = the reduction's quotient digits), we get N R^-1 = N (R^-1 mod N)
(mod N^2) and therefore

    X Y R^-1 = t + N * REDC_N(x0 y1 + x1 y0 - m)          (mod N^2)

i.e. the Montgomery product modulo N^2 is two interleaved Montgomery products modulo N
that share their row loop: the t part reduces x0*y0 and hands its quotient digit q_i of
row i straight to the s part, which adds (K'_i - q_i) in that row's retiring column.
-m is taken as (R - 1 - m) + K with K = (1 - R) mod N, so every column stays non-negative:
K'_i = (2^29 - 1) + K_i (host constants, the group engines' K' too).  Per product 36 rows x
(36 + 36 + 72 + 36 + 1) + 68 (the mid-product reduction) = 6 584 v_mad_u64_u32 (square,
triangular: 4 658) -- 4 % fewer than with 37 limbs of 28 bits (rounds 1-3: 6 882 / 4 847).

Bounds (N < 2^1024, R = 2^1044 >= 2^20 N): digits < 2N in -> digits < 2N out.  A digit up to
R - 1 in one operand (the hash h < 2^1044 entering as (h, 0), the plaintext digit of
N*pt + 1 = (1, pt)) gives digits < 3N + 1, which the next product brings back below 2N.
Columns: a row adds at most 2^59 (a doubled cross product, or x0 y1 + x1 y0) + 2^58 (q N) to a
slot, so 36 rows could pass 2^64; after row 17 every slot but the youngest hands its high dword
to the slot above (x 8 = 2^32 / 2^29) and keeps the low one -- each column then gathers at most
19 rows' products from below 2^36: 19 * 1.5 * 2^59 + 2^58 + 2^36 < 2^64 (the simulator asserts
it on every multiply).

Register plan (per lane, wave64):
  v[2k:2k+1]      k=0..34  t-window accumulators At_k (64-bit)
  v[70+2k:71+2k]  k=0..34  s-window accumulators As_k
  v140..v175      B digit 0 limbs b0_j
  v176..v211      B digit 1 limbs b1_j
  v212, v213      x0_i, x1_i of the current row;  v214, v215 the next row's (prefetch)
  v[216:217]      Tt = retiring column of the t part;  v[218:219] Ts (s part)
  v220 q, v221 q', v222 np = -N^-1 mod 2^29, v223 LDS address of x0_i, v224 scratch,
  v225 K'_i - q
  s20..s29, s36..s61   N_0..N_9, N_10..N_35 (uniform, loaded once per product)
  s62..s97             K'_0..K'_35 (row i reads K'_i by s_movrels with m0 = i)
  s34 row counter, s35 K'_i;  vcc: unused carry-out of v_mad_u64_u32;  scc clobbered;
  m0 (reserved to the compiler) saved in s19 on entry and restored on exit.

Operands: A is the lane's LDS column (limb k of the 72 at byte a_off + k*1024: rows 0..35
digit 0, rows 36..71 digit 1; the last row's prefetch reads row 72) and receives the result;
B comes from global memory (uniform base + per-lane byte offset, limb stride 1024 B: the
workgroup-blocked layout of tables and residue columns) or, for the square, from the A
column itself.  The constants block (80 words, FBM_CST_NA29 in fbm_internal.hpp) holds
N_0..N_9 at words 0..9, N_10..N_35 at words 16..41 and K'_0..K'_35 at words 42..77.

Usage:  python tools/gen_nadic_asm.py   (rewrites the header; the build does not run this)
"""

import os

LB = 29     # bits per limb
L = 36      # limbs per digit (R = 2^(LB L) = 2^1044)
NW = L - 1  # window accumulators per part
MID = 18    # rows before the mid-product reduction
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "fedbiomed_amd", "csrc", "fbm_nadic_asm.hpp")
MASK = hex((1 << LB) - 1)
AS0 = 2 * NW            # s window of the general product
B00, B10 = 2 * AS0, 2 * AS0 + L


def At(k):
    return f"v[{2 * k}:{2 * k + 1}]"


def AtLo(k):
    return f"v{2 * k}"


def AtHi(k):
    return f"v{2 * k + 1}"


def As(k):
    return f"v[{AS0 + 2 * k}:{AS0 + 2 * k + 1}]"


def AsLo(k):
    return f"v{AS0 + 2 * k}"


def AsHi(k):
    return f"v{AS0 + 2 * k + 1}"


def B0(j):
    return f"v{B00 + j}"


def B1(j):
    return f"v{B10 + j}"


def Ns(j):
    return f"s{20 + j}" if j < 10 else f"s{36 + j - 10}"


KBASE = f"s{36 + L - 10}"  # K'_0 right after N_35
_X = B10 + L
X0, X1, X0N, X1N = f"v{_X}", f"v{_X + 1}", f"v{_X + 2}", f"v{_X + 3}"
TT, TTLO, TS, TSLO = f"v[{_X + 4}:{_X + 5}]", f"v{_X + 4}", f"v[{_X + 6}:{_X + 7}]", f"v{_X + 6}"
Q, Q2, NPV, AADR, TMP, CQ = (f"v{_X + 8 + i}" for i in range(6))
MM_NREG = _X + 14
ROW1 = L * 1024  # byte offset of digit 1 in the LDS column


def load_consts():
    return [
        "s_load_dwordx8 s[20:27], %[NK], 0x0",
        "s_load_dwordx2 s[28:29], %[NK], 0x20",
        "s_load_dwordx16 s[36:51], %[NK], 0x40",
        "s_load_dwordx16 s[52:67], %[NK], 0x80",
        "s_load_dwordx16 s[68:83], %[NK], 0xc0",
        "s_load_dwordx16 s[84:99], %[NK], 0x100",
    ]


def breg(j):
    return B0(j) if j < L else B1(j - L)


def load_b_global():
    # the caller may just have stored this column (same lane): drain stores before loading
    out = ["s_waitcnt vmcnt(0)", f"v_mov_b32 {TMP}, %[b]"]
    for j in range(2 * L):
        if j and j % 4 == 0:
            out.append(f"v_add_u32 {TMP}, 0x1000, {TMP}")
        out.append(f"global_load_dword {breg(j)}, {TMP}, %[bb] offset:{(j % 4) * 1024}")
    return out


def load_b_nude():
    """The encrypt's last operand nude = N pt + 1 = the digit pair (1, pt): digit 0 as immediates, only
    digit 1's rows from global (jl_nude_kernel stores 36 rows per ciphertext block, not 72)."""
    out = ["s_waitcnt vmcnt(0)", f"v_mov_b32 {TMP}, %[b]"]
    for j in range(L):
        if j and j % 4 == 0:
            out.append(f"v_add_u32 {TMP}, 0x1000, {TMP}")
        out.append(f"global_load_dword {breg(L + j)}, {TMP}, %[bb] offset:{(j % 4) * 1024}")
    out += [f"v_mov_b32 {breg(j)}, {1 if j == 0 else 0}" for j in range(L)]
    return out


def load_b_square():
    out = [f"v_add_u32 {TMP}, 0x10000, %[a]"]
    for j in range(2 * L):
        if j < 64:
            out.append(f"ds_read_b32 {breg(j)}, %[a] offset:{j * 1024}")
        else:
            out.append(f"ds_read_b32 {breg(j)}, {TMP} offset:{(j - 64) * 1024}")
    out.append("s_waitcnt lgkmcnt(0)")
    out += [f"v_lshlrev_b32 {B1(j)}, 1, {B1(j)}" for j in range(L)]
    return out


def row(first, sq):
    """One row i of the fused t/s product.  x0_i (and x1_i) are in X0 (X1); s35 = K'_i."""
    out = [f"ds_read_b32 {X0N}, {AADR} offset:1024"]
    if not sq:
        out.append(f"ds_read_b32 {X1N}, {AADR} offset:{ROW1 + 1024}")
    kreg = KBASE if first else "s35"
    # ---- t part: x0_i * b0, quotient q, q * N ----
    out.append(f"v_mad_u64_u32 {TT}, vcc, {X0}, {B0(0)}, {'0' if first else At(0)}")
    for j in range(1, L):
        addend = "0" if (first or j == NW) else At(j)
        out.append(f"v_mad_u64_u32 {At(j - 1)}, vcc, {X0}, {B0(j)}, {addend}")
        if j == 3:
            out.append(f"v_mul_lo_u32 {Q}, {TTLO}, {NPV}")
        if j == 6:
            out.append(f"v_and_b32 {Q}, {MASK}, {Q}")
        if j == 8:
            out.append(f"v_sub_u32 {CQ}, {kreg}, {Q}")  # K'_i - q_i  (>= 0: K'_i >= 2^29 - 1)
    out.append(f"v_mad_u64_u32 {TT}, vcc, {Q}, {Ns(0)}, {TT}")
    for j in range(1, L):
        out.append(f"v_mad_u64_u32 {At(j - 1)}, vcc, {Q}, {Ns(j)}, {At(j - 1)}")
    # ---- s part: x0_i * b1 (+ x1_i * b0), + (K'_i - q_i), quotient q', q' * N ----
    out.append(f"v_mad_u64_u32 {TS}, vcc, {X0}, {B1(0)}, {'0' if first else As(0)}")
    for j in range(1, L):
        addend = "0" if (first or j == NW) else As(j)
        out.append(f"v_mad_u64_u32 {As(j - 1)}, vcc, {X0}, {B1(j)}, {addend}")
        if j == 12:
            out.append(f"v_mad_u64_u32 {TS}, vcc, {CQ}, 1, {TS}")
        if not sq and j == 24:
            out.append(f"v_mad_u64_u32 {TS}, vcc, {X1}, {B0(0)}, {TS}")
        if sq and j == 20:
            out.append(f"v_mul_lo_u32 {Q2}, {TSLO}, {NPV}")
        if sq and j == 26:
            out.append(f"v_and_b32 {Q2}, {MASK}, {Q2}")
    if not sq:
        for j in range(1, L):
            out.append(f"v_mad_u64_u32 {As(j - 1)}, vcc, {X1}, {B0(j)}, {As(j - 1)}")
            if j == 3:
                out.append(f"v_mul_lo_u32 {Q2}, {TSLO}, {NPV}")
            if j == 6:
                out.append(f"v_and_b32 {Q2}, {MASK}, {Q2}")
    out.append(f"v_mad_u64_u32 {TS}, vcc, {Q2}, {Ns(0)}, {TS}")
    for j in range(1, L):
        out.append(f"v_mad_u64_u32 {As(j - 1)}, vcc, {Q2}, {Ns(j)}, {As(j - 1)}")
    # ---- retire column i of both parts ----
    out += [f"v_lshrrev_b64 {TT}, {LB}, {TT}", f"v_lshl_add_u64 {At(0)}, {TT}, 0, {At(0)}",
            f"v_lshrrev_b64 {TS}, {LB}, {TS}", f"v_lshl_add_u64 {As(0)}, {TS}, 0, {As(0)}",
            f"v_add_u32 {AADR}, 0x400, {AADR}", "s_waitcnt lgkmcnt(0)", f"v_mov_b32 {X0}, {X0N}"]
    if not sq:
        out.append(f"v_mov_b32 {X1}, {X1N}")
    return out


def mid_reduce(pairs, keep=None, one=None):
    """After row MID - 1: every slot (pair lo register) but the youngest keeps its low dword and
    hands the high one to the slot above (x 8 = 2^32 / 2^29).  `pairs`: per part, the window's
    slot pair low registers from the oldest column to the youngest.  `keep`: per part, the slot
    indices that need the reduction (None: all) -- the others' columns provably stay below 2^64
    without it (tests/asm_bounds.py).  `one`: per part, slots whose high dword is set to 1 instead
    of 0 (the column keeps 2^32 + its low dword: it stays >= 2^32 > any quotient digit a later row
    subtracts from it; the 2^32 so added per such column is a constant the host cancels in the
    s window's initial pairs -- sq_kfold_extra)."""
    chains = []
    for part, regs in enumerate(pairs):
        ch = []
        for k in range(len(regs) - 1):
            if keep is not None and k not in keep[part]:
                continue
            lo, nxt = regs[k], regs[k + 1]
            hi = f"v{int(lo[1:]) + 1}"
            hv = 1 if one is not None and k in one[part] else 0
            ch += [f"v_mad_u64_u32 v[{nxt[1:]}:{int(nxt[1:]) + 1}], vcc, {hi}, 8, v[{nxt[1:]}:{int(nxt[1:]) + 1}]",
                   f"v_mov_b32 {hi}, {hv}"]
        chains.append(ch)
    out = []
    for k in range(max(len(c) for c in chains)):
        for ch in chains:
            if k < len(ch):
                out.append(ch[k])
    return out


def normalise_store():
    out = [f"v_add_u32 {TMP}, 0x10000, %[a]"]

    def st(k, reg):
        if k < 64:
            return f"ds_write_b32 %[a], {reg} offset:{k * 1024}"
        return f"ds_write_b32 {TMP}, {reg} offset:{(k - 64) * 1024}"

    for acc, lo, carry, carry_lo, base in ((At, AtLo, TT, TTLO, 0), (As, AsLo, TS, TSLO, L)):
        out += [f"v_lshrrev_b64 {carry}, {LB}, {acc(0)}", f"v_and_b32 {lo(0)}, {MASK}, {lo(0)}", st(base, lo(0))]
        for k in range(1, NW):
            out += [f"v_lshl_add_u64 {acc(k)}, {carry}, 0, {acc(k)}",
                    f"v_lshrrev_b64 {carry}, {LB}, {acc(k)}",
                    f"v_and_b32 {lo(k)}, {MASK}, {lo(k)}",
                    st(base + k, lo(k))]
        out.append(st(base + NW, carry_lo))
    out.append("s_waitcnt lgkmcnt(0)")
    return out


M0_SAVE = "s19"  # m0 is reserved to the compiler: saved here (declared clobbered) and restored
CARRY_PAIRS = ("vcc", "s[16:17]")  # the mads' (never read) carry-outs, alternated


def rotate_carries(lines, pairs=CARRY_PAIRS):
    """Alternate the carry-out destination of successive v_mad_u64_u32 over `pairs`: mads that all
    write vcc chain through it (write-after-write) and a wave issues one every ~8.8 clocks, two pairs
    in turn ~5.8 (tools/microbench/gen_oprate.py).  Every mad stays 8 bytes (the computed jumps)."""
    out, i = [], 0
    for ln in lines:
        if ln.startswith(("v_mad_u64_u32", "v_mad_i64_i32")) and ", vcc," in ln:
            ln = ln.replace(", vcc,", f", {pairs[i % len(pairs)]},", 1)
            i += 1
        out.append(ln)
    return out


def product(sq, nude=False):
    body = [f"s_mov_b32 {M0_SAVE}, m0"] + load_consts()
    body += load_b_square() if sq else (load_b_nude() if nude else load_b_global())
    body += [f"v_mov_b32 {NPV}, %[np]", f"v_mov_b32 {AADR}, %[a]", f"ds_read_b32 {X0}, {AADR}"]
    if not sq:
        body.append(f"ds_read_b32 {X1}, {AADR} offset:{ROW1}")
    body += ["s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body += row(True, sq)
    # s_movrels after an SALU write of m0 needs a wait state (the hazard is not checked in asm)
    body += ["s_mov_b32 s34, 1", "1:", "s_mov_b32 m0, s34", "s_nop 1", f"s_movrels_b32 s35, {KBASE}"]
    body += row(False, sq)
    body += [f"s_cmp_lg_u32 s34, {MID - 1}", "s_cbranch_scc1 2f"]
    body += mid_reduce([[AtLo(k) for k in range(NW)], [AsLo(k) for k in range(NW)]]) + ["2:"]
    body += ["s_add_u32 s34, s34, 1", f"s_cmp_lg_u32 s34, {L}", "s_cbranch_scc1 1b"]
    body += normalise_store()
    body += [f"s_mov_b32 m0, {M0_SAVE}", "s_nop 1"]  # m0 read right after the asm: wait state
    return rotate_carries(body)


# ------------------------------------------------------------------------------------------
# Squaring with a triangular t part: X^2 = x0^2 + N (2 x0 x1), and x0^2 needs each cross
# product x0_i x0_k (i < k) once, doubled, plus the diagonals x0_h^2.  Row i adds
# 2 x0_i x0_k for k > i -- a contiguous suffix of the row's t multiply sequence, entered by
# a computed jump (s_setpc_b64; every entry is one 8-byte v_mad_u64_u32) -- and, for even i,
# the diagonal x0_{i/2}^2 of column i (read from the LDS column along a running address:
# rows are unrolled in odd/even pairs so the parity is static).  Diagonals of columns 36..70
# are added after the loop from the B registers.  The t products are added in place
# (At_k, k = window position) and the q*N pass shifts the window, so the t window has 36
# pairs (At_35 is written, not accumulated, by each row's last cross product).  Column i is
# complete when its quotient is taken: cross products of column i come from rows < i, the
# diagonal from row i itself.  The s part runs full rows of (2 x0_i) * x1 (the doubled row
# operand serves both parts).  Column bounds as the general product's (the mid-product
# reduction after row 17, inside the row-pair loop).
# Register plan: At_k v[2k:2k+1] (k=0..35), As_k v[72+2k:73+2k] (k=0..34), b0 = x0
# v142..v177, b1 = x1 v178..v213, x0_0 v214, next x0 v215, 2 x0_i v216, Tt v[218:219],
# Ts v[220:221], q v222, q' v223, np v224, LDS address v225, scratch v226, K'_i - q v227,
# diagonal limb v228, its LDS address v229;  s[30:31] jump target, s34 row, s35 K'_i / offset.
# ------------------------------------------------------------------------------------------
SAS0 = 2 * L                  # s window of the square
SB00 = SAS0 + 2 * NW
SB10 = SB00 + L
_SX = SB10 + L


def SAt(k):
    return f"v[{2 * k}:{2 * k + 1}]"


def SAtLo(k):
    return f"v{2 * k}"


def SAs(k):
    return f"v[{SAS0 + 2 * k}:{SAS0 + 2 * k + 1}]"


def SAsLo(k):
    return f"v{SAS0 + 2 * k}"


def SB0(j):
    return f"v{SB00 + j}"


def SB1(j):
    return f"v{SB10 + j}"


SX0, SX0N, SX0D = f"v{_SX}", f"v{_SX + 1}", f"v{_SX + 2}"
_ST = _SX + 3 + (_SX + 3) % 2  # 64-bit pairs start on an even VGPR
STT, STTLO, STS, STSLO = f"v[{_ST}:{_ST + 1}]", f"v{_ST}", f"v[{_ST + 2}:{_ST + 3}]", f"v{_ST + 2}"
SQ, SQ2, SNPV, SAADR, STMP, SCQ, SDI, SDADDR = (f"v{_ST + 4 + i}" for i in range(8))
SQ_NREG = _ST + 12


def sq_tri(tag, first=False):
    """Doubled cross products 2 x0_i x0_k, k = 1..L-1 (entered at k = i + 1 by the jump;
    whole, with addend 0, for row 0).  k = L-1 writes: the shift consumed the old top."""
    out = [f"v_mad_u64_u32 {SAt(k)}, vcc, {SX0D}, {SB0(k)}, {'0' if first else SAt(k)}" for k in range(1, L - 1)]
    out.append(f"v_mad_u64_u32 {SAt(L - 1)}, vcc, {SX0D}, {SB0(L - 1)}, 0")
    return out


def sq_jump(tag, offset_expr):
    """s[30:31] <- address of the tri-block entry k = i + 1 (byte offset 8 i, in s35)."""
    return offset_expr + ["s_getpc_b64 s[30:31]",
                          f".Lfbm_na_pc{tag}_%=:",
                          "s_add_u32 s30, s30, s35",
                          "s_addc_u32 s31, s31, 0",
                          f"s_add_u32 s30, s30, .Lfbm_na_tri{tag}_%= - .Lfbm_na_pc{tag}_%=",
                          "s_addc_u32 s31, s31, 0",
                          "s_setpc_b64 s[30:31]",
                          f".Lfbm_na_tri{tag}_%=:"]


def sq_row(kind, kreg="s35"):
    """kind: 'first' (row 0), 'odd', 'even' (loop rows), 'last' (row L - 1 = 35: odd, no cross
    products).  On entry X0 = x0_i; s35 = K'_i (kreg)."""
    first = kind == "first"
    even = kind in ("first", "even")
    out = [f"ds_read_b32 {SX0N}, {SAADR} offset:1024"]
    if even:  # diagonal x0_{i/2}^2 of column i (DI holds it), then prefetch the next even row's
        out.append(f"v_mad_u64_u32 {SAt(0)}, vcc, {SDI}, {SDI}, {'0' if first else SAt(0)}")
        out += [f"v_add_u32 {SDADDR}, 0x400, {SDADDR}", f"ds_read_b32 {SDI}, {SDADDR}"]
    out.append(f"v_mul_lo_u32 {SQ}, {SAtLo(0)}, {SNPV}")  # column i is complete
    # ---- s part: (2 x0_i) * x1, + (K'_i - q), q' ----
    out.append(f"v_mad_u64_u32 {STS}, vcc, {SX0D}, {SB1(0)}, {'0' if first else SAs(0)}")
    for j in range(1, L):
        addend = "0" if (first or j == NW) else SAs(j)
        out.append(f"v_mad_u64_u32 {SAs(j - 1)}, vcc, {SX0D}, {SB1(j)}, {addend}")
        if j == 2:
            out.append(f"v_and_b32 {SQ}, {MASK}, {SQ}")
        if j == 4:
            out.append(f"v_sub_u32 {SCQ}, {kreg}, {SQ}")
        if j == 12:
            out.append(f"v_mad_u64_u32 {STS}, vcc, {SCQ}, 1, {STS}")
        if j == 20:
            out.append(f"v_mul_lo_u32 {SQ2}, {STSLO}, {SNPV}")
        if j == 26:
            out.append(f"v_and_b32 {SQ2}, {MASK}, {SQ2}")
    # ---- t part: doubled cross products (suffix k > i) ----
    if first:
        out += sq_tri("0", first=True)
    elif kind == "odd":
        out += sq_jump("o", ["s_lshl_b32 s35, s34, 3"]) + sq_tri("o")
    elif kind == "even":
        out += sq_jump("e", ["s_add_u32 s35, s34, 1", "s_lshl_b32 s35, s35, 3"]) + sq_tri("e")
    # ---- t: q * N (shifting the window);  s: q' * N ----
    top = "0" if kind == "last" else SAt(L - 1)
    out.append(f"v_mad_u64_u32 {STT}, vcc, {SQ}, {Ns(0)}, {SAt(0)}")
    for k in range(1, L):
        out.append(f"v_mad_u64_u32 {SAt(k - 1)}, vcc, {SQ}, {Ns(k)}, {SAt(k) if k < L - 1 else top}")
    out.append(f"v_mad_u64_u32 {STS}, vcc, {SQ2}, {Ns(0)}, {STS}")
    for j in range(1, L):
        out.append(f"v_mad_u64_u32 {SAs(j - 1)}, vcc, {SQ2}, {Ns(j)}, {SAs(j - 1)}")
    out += [f"v_lshrrev_b64 {STT}, {LB}, {STT}", f"v_lshl_add_u64 {SAt(0)}, {STT}, 0, {SAt(0)}",
            f"v_lshrrev_b64 {STS}, {LB}, {STS}", f"v_lshl_add_u64 {SAs(0)}, {STS}, 0, {SAs(0)}",
            f"v_add_u32 {SAADR}, 0x400, {SAADR}", "s_waitcnt lgkmcnt(0)", f"v_lshlrev_b32 {SX0D}, 1, {SX0N}"]
    return out


def krow(row_expr):
    """m0 <- row index, then s35 <- K'_row (s_movrels needs a wait state after the m0 write)."""
    return row_expr + ["s_nop 1", f"s_movrels_b32 s35, {KBASE}"]


def square_tri():
    body = [f"s_mov_b32 {M0_SAVE}, m0"] + load_consts()
    body.append(f"v_add_u32 {STMP}, 0x10000, %[a]")
    for j in range(2 * L):
        reg = SB0(j) if j < L else SB1(j - L)
        if j < 64:
            body.append(f"ds_read_b32 {reg}, %[a] offset:{j * 1024}")
        else:
            body.append(f"ds_read_b32 {reg}, {STMP} offset:{(j - 64) * 1024}")
    body += [f"v_mov_b32 {SNPV}, %[np]", f"v_mov_b32 {SAADR}, %[a]", f"ds_read_b32 {SX0}, %[a]",
             f"ds_read_b32 {SDI}, %[a]", f"v_mov_b32 {SDADDR}, %[a]", "s_waitcnt lgkmcnt(0)",
             f"v_lshlrev_b32 {SX0D}, 1, {SX0}"]
    assert L % 2 == 0 and (MID - 1) % 2 == 1  # rows 1 .. L-2 in (odd, even) pairs, row L-1 peeled
    body += sq_row("first", kreg=KBASE)
    body += ["s_mov_b32 s34, 1", "1:"]
    body += krow(["s_mov_b32 m0, s34"]) + sq_row("odd")
    # after row MID - 1 (odd): the mid-product reduction (the t window's top pair is dead here --
    # the next row's last cross product writes it -- and the s window's youngest is kept)
    body += [f"s_cmp_lg_u32 s34, {MID - 1}", "s_cbranch_scc1 2f"]
    body += mid_reduce([[SAtLo(k) for k in range(L - 1)], [SAsLo(k) for k in range(NW)]]) + ["2:"]
    body += krow(["s_add_u32 m0, s34, 1"]) + sq_row("even")
    body += ["s_add_u32 s34, s34, 2", f"s_cmp_lg_u32 s34, {L - 1}", "s_cbranch_scc1 1b"]
    body += krow([f"s_mov_b32 m0, {L - 1}"]) + sq_row("last")
    # diagonals of columns L .. 2L-2 (h >= L/2): column 2h sits at window position 2h - L
    body += [f"v_mad_u64_u32 {SAt(2 * h - L)}, vcc, {SB0(h)}, {SB0(h)}, {SAt(2 * h - L)}" for h in range(L // 2, L)]
    body.append(f"v_add_u32 {STMP}, 0x10000, %[a]")

    def st(k, reg):
        if k < 64:
            return f"ds_write_b32 %[a], {reg} offset:{k * 1024}"
        return f"ds_write_b32 {STMP}, {reg} offset:{(k - 64) * 1024}"

    for acc, lo, carry, carry_lo, base in ((SAt, SAtLo, STT, STTLO, 0), (SAs, SAsLo, STS, STSLO, L)):
        body += [f"v_lshrrev_b64 {carry}, {LB}, {acc(0)}", f"v_and_b32 {lo(0)}, {MASK}, {lo(0)}", st(base, lo(0))]
        for k in range(1, NW):
            body += [f"v_lshl_add_u64 {acc(k)}, {carry}, 0, {acc(k)}",
                     f"v_lshrrev_b64 {carry}, {LB}, {acc(k)}",
                     f"v_and_b32 {lo(k)}, {MASK}, {lo(k)}",
                     st(base + k, lo(k))]
        body.append(st(base + NW, carry_lo))
    body += ["s_waitcnt lgkmcnt(0)", f"s_mov_b32 m0, {M0_SAVE}", "s_nop 1"]
    return rotate_carries(body)


# ------------------------------------------------------------------------------------------
# Product by the SHORT base h < 2^(29 KS) (one FDH digest: 256 bits, KS = 9 limbs) -- the
# multiply of the binary exponentiation (jl_exp_kernel's short path).  The multiplier rows are
# h's KS limbs (digit 1 = 0), B = the running value X from the lane's own LDS column, and the
# Montgomery reduction takes KS quotient digits only:
#     X h 2^-(29 KS)  (mod N^2)  =  t + N s,
#     t = (x0 h + m N) / 2^(29 KS)                        (m = sum q_i 2^(29 i), i < KS)
#     s = (x1 h + (2^(29 KS) - m) + D + m' N) / 2^(29 KS),   D = N - 2^(29 KS)
# -- 2^(29 KS) - m is the rows' retiring-column adds (2^29 - 1 - q_i, + 1 in row 0), D enters as
# the s window's initial value (row 0's addends: pairs (D_j, 0) read from LDS), so the s
# numerator is x1 h - m + N (= x1 h - m mod N, and >= 0: m < 2^(29 KS) < N).  KS (36 + 36 +
# 36 + 36 + 1) = 1 305 multiplies against 6 584 for a general product, and no table.  Bounds
# (N > 2^(29 KS)): digits < 2N in -> t < 3N, s < 3N + 2 (the next squaring brings them back
# below 2N); a column gathers at most KS rows of 2 products < 2^58: < 2^62.2, no mid-product
# reduction.  The factor 2^-(29 KS) per multiply (and R^-1 per squaring) is a constant of the
# exponent, cancelled by one product with a host-built constant after the chain.
# Register plan: the general product's, with h's limbs in v226..v234 and (D_35, 0) in v[214:215]
# (the row-operand prefetch registers, unused here); the multiplier needs no LDS rows.
# ------------------------------------------------------------------------------------------
KS = 9
SHORT_LOOPED = True   # rows 1..8 as a loop (3 KB of code instead of 14 KB: the unrolled square is 43 KB)
HS = [f"v{MM_NREG + i}" for i in range(KS)]
D35 = f"v[{_X + 2}:{_X + 3}]"
HADDR = X1  # (looped rows) the address of the next row's limb of h
MS_NREG = MM_NREG if SHORT_LOOPED else MM_NREG + KS


def short_row(i, x=None):
    """Row i of the short product: multiplier limb h_i (HS[i], or the register x), t then s part,
    both retires (rows >= 1 are the same instruction stream whatever i: the loop body)."""
    x, first = (x or HS[i]), i == 0
    out = [f"v_mad_u64_u32 {TT}, vcc, {x}, {B0(0)}, {'0' if first else At(0)}"]
    for j in range(1, L):
        addend = "0" if (first or j == NW) else At(j)
        out.append(f"v_mad_u64_u32 {At(j - 1)}, vcc, {x}, {B0(j)}, {addend}")
        if j == 3:
            out.append(f"v_mul_lo_u32 {Q}, {TTLO}, {NPV}")
        if j == 6:
            out.append(f"v_and_b32 {Q}, {MASK}, {Q}")
        if j == 8 and not SHORT_KFOLD:  # 2^29 - 1 - q_i (+ 1 in row 0: the sum over the rows is 2^(29 KS) - m)
            out.append(f"v_sub_u32 {CQ}, {hex(1 << LB) if first else MASK}, {Q}")
    out.append(f"v_mad_u64_u32 {TT}, vcc, {Q}, {Ns(0)}, {TT}")
    for j in range(1, L):
        out.append(f"v_mad_u64_u32 {At(j - 1)}, vcc, {Q}, {Ns(j)}, {At(j - 1)}")
    # s part: the window's addends (row 0: D, loaded into it; the top slot's D_35 from D35)
    out.append(f"v_mad_u64_u32 {TS}, vcc, {x}, {B1(0)}, {As(0)}")
    for j in range(1, L):
        addend = (D35 if first else "0") if j == NW else As(j)
        out.append(f"v_mad_u64_u32 {As(j - 1)}, vcc, {x}, {B1(j)}, {addend}")
        if j == 12:
            out.append(f"v_mad_i64_i32 {TS}, vcc, {Q}, -1, {TS}" if SHORT_KFOLD else
                       f"v_mad_u64_u32 {TS}, vcc, {CQ}, 1, {TS}")
        if j == 20:
            out.append(f"v_mul_lo_u32 {Q2}, {TSLO}, {NPV}")
        if j == 26:
            out.append(f"v_and_b32 {Q2}, {MASK}, {Q2}")
    out.append(f"v_mad_u64_u32 {TS}, vcc, {Q2}, {Ns(0)}, {TS}")
    for j in range(1, L):
        out.append(f"v_mad_u64_u32 {As(j - 1)}, vcc, {Q2}, {Ns(j)}, {As(j - 1)}")
    out += [f"v_lshrrev_b64 {TT}, {LB}, {TT}", f"v_lshl_add_u64 {At(0)}, {TT}, 0, {At(0)}",
            f"v_lshrrev_b64 {TS}, {LB}, {TS}", f"v_lshl_add_u64 {As(0)}, {TS}, 0, {As(0)}"]
    return out


# Round 4: the short product with h's KS limbs in registers (asm inputs %[h0] .. %[h8], held by the
# kernel for the whole chain: no global reads of h per product) and its rows unrolled; the rows'
# 2^29 - 1 - q_i folded like the square's K': the s window starts at the pairs (D'_j, 0),
# D'_j = D_j + (2^29 - 1) [j < KS] + [j == 0] -- a non-normalised N (D + 2^261) -- and each row
# subtracts q_i with one v_mad_i64_i32 (column i >= 2^29 - 1 >= q_i).
SHORT_KFOLD = True


def mul_short_reg():
    body = list(load_consts())
    body.append(f"v_add_u32 {AADR}, 0x10000, %[a]")
    for j in range(2 * L):
        if j < 64:
            body.append(f"ds_read_b32 {breg(j)}, %[a] offset:{j * 1024}")
        else:
            body.append(f"ds_read_b32 {breg(j)}, {AADR} offset:{(j - 64) * 1024}")
    body += [f"ds_read_b64 {As(j)}, %[d] offset:{8 * j}" for j in range(NW)]
    body += [f"ds_read_b64 {D35}, %[d] offset:{8 * NW}", f"v_mov_b32 {NPV}, %[np]", "s_waitcnt lgkmcnt(0)"]
    for i in range(KS):
        body += short_row(i, f"%[h{i}]")
    body += normalise_store()
    return rotate_carries(body)


def mul_short():
    body = list(load_consts())
    # h's KS limbs: global, workgroup-blocked (limb k at hb + h_off + k * 1024)
    body += ["s_waitcnt vmcnt(0)", f"v_mov_b32 {TMP}, %[h]"]
    if SHORT_LOOPED:  # limb 0 now, each next one prefetched a row ahead (HADDR = its address)
        body += [f"global_load_dword {X0}, {TMP}, %[hb]", f"v_add_u32 {HADDR}, 0x400, {TMP}"]
    else:
        for k in range(KS):
            if k and k % 4 == 0:
                body.append(f"v_add_u32 {TMP}, 0x1000, {TMP}")
            body.append(f"global_load_dword {HS[k]}, {TMP}, %[hb] offset:{(k % 4) * 1024}")
    # B = X from the lane's column (undoubled); the s window <- (D_j, 0), D35 <- (D_35, 0)
    body.append(f"v_add_u32 {AADR}, 0x10000, %[a]")
    for j in range(2 * L):
        if j < 64:
            body.append(f"ds_read_b32 {breg(j)}, %[a] offset:{j * 1024}")
        else:
            body.append(f"ds_read_b32 {breg(j)}, {AADR} offset:{(j - 64) * 1024}")
    body += [f"ds_read_b64 {As(j)}, %[d] offset:{8 * j}" for j in range(NW)]
    body += [f"ds_read_b64 {D35}, %[d] offset:{8 * NW}", f"v_mov_b32 {NPV}, %[np]",
             "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    if SHORT_LOOPED:  # row 0 peeled, rows 1 .. KS-1 a runtime loop over row pairs (operands X0N / X0)
        assert (KS - 1) % 2 == 0

        def pref(dst):  # the next row's limb of h, a row ahead
            return [f"global_load_dword {dst}, {HADDR}, %[hb]", f"v_add_u32 {HADDR}, 0x400, {HADDR}"]

        xb = AADR  # the second operand register (AADR is free once the prologue's loads are in; X0N
        #            holds D_35 until row 0's last s product)
        body += pref(xb) + short_row(0, X0) + ["s_waitcnt vmcnt(0)"]
        body += ["s_mov_b32 s34, 0", "3:"]
        body += pref(X0) + short_row(1, xb) + ["s_waitcnt vmcnt(0)"]
        body += pref(xb) + short_row(1, X0) + ["s_waitcnt vmcnt(0)"]
        body += ["s_add_u32 s34, s34, 1", f"s_cmp_lg_u32 s34, {(KS - 1) // 2}", "s_cbranch_scc1 3b"]
    else:
        for i in range(KS):
            body += short_row(i)
    body += normalise_store()
    return rotate_carries(body)


def ms_mads():
    return KS * (4 * L + 1)


# ------------------------------------------------------------------------------------------
# The triangular square with every row unrolled (round 3): the same arithmetic, registers and
# instruction order per row as square_tri, but with the row index static -- the cross products
# k = i + 1 .. 35 emitted directly (no computed jump, s_setpc's instruction-buffer refetch), K'_i
# read from s(62 + i) (no m0 / s_movrels), the diagonal x_(i/2)^2 of an even row from the B
# register that holds x_(i/2) (no LDS read, no address add), the row operands read at static
# offsets from the column base (no address add).  4 273 instructions (~35 KB) instead of a loop;
# bit-identical results (tests/test_nadic_asm.py runs both).
# ------------------------------------------------------------------------------------------
UNROLLED_SQUARE = True
# Round 4: (1) K' folded -- the s window starts at the pairs (K'_j, 0) (LDS, %[k]) and each row
# subtracts its quotient digit with one v_mad_i64_i32 (q * -1 + column; the column holds K'_i >= 2^29 - 1
# >= q, so it stays non-negative) instead of v_sub (K'_i - q) + v_mad_u64_u32 (+ 1 x (K'_i - q)): one VALU
# instruction less per row; (2) the mid-product reduction only on the slots whose columns could
# otherwise pass 2^64 (tests/asm_bounds.py proves the rest stay below it for every operand within the
# product's input bounds: 6 t slots and 28 s slots of 34 + 34).
SQ_KFOLD = True
SQ_MID_KEEP = (set(range(14, 20)), set(range(3, 31)))  # (t slots, s slots); None: every slot
SQ_MID_T = SQ_MID_S = MID  # the reduction follows row SQ_MID_{T,S} - 1 (t part, s part)


def sq_one_slots():
    """The s slots the mid-product reduction leaves at 2^32 + low dword (mid_reduce's `one`): those
    reduced whose column (SQ_MID_S + slot) still has a quotient digit to lose (column <= L - 1)."""
    keep = range(NW - 1) if SQ_MID_KEEP is None else SQ_MID_KEEP[1]
    return {k for k in keep if SQ_MID_S + k <= L - 1}


def sq_kfold_extra():
    """E: what the reduction's high dwords of 1 add to the square's s numerator, sum over those slots
    of 2^(32 + 29 column).  The host's initial pairs are (2^29 - 1 + P'_j, 0) with P' = (K - E) mod N, so
    that the constant added in all is R - 1 + P' + E == 0 (mod N) (K = (1 - R) mod N)."""
    return sum(1 << (32 + LB * (SQ_MID_S + k)) for k in sq_one_slots()) if SQ_KFOLD else 0


def sq_row_static(i):
    first, last, even = i == 0, i == L - 1, i % 2 == 0
    kreg = f"s{62 + i}"  # K'_i (KBASE + i)
    out = [] if last else [f"ds_read_b32 {SX0N}, %[a] offset:{(i + 1) * 1024}"]
    if even:  # the diagonal x0_(i/2)^2 of column i completes it
        out.append(f"v_mad_u64_u32 {SAt(0)}, vcc, {SB0(i // 2)}, {SB0(i // 2)}, {'0' if first else SAt(0)}")
    out.append(f"v_mul_lo_u32 {SQ}, {SAtLo(0)}, {SNPV}")
    # ---- s part: (2 x0_i) * x1, - q (K'_i pre-added to column i: SQ_KFOLD) or + (K'_i - q), q' ----
    s0 = (STS if SQ_KFOLD else "0") if first else SAs(0)
    out.append(f"v_mad_u64_u32 {STS}, vcc, {SX0D}, {SB1(0)}, {s0}")
    for j in range(1, L):
        if first:
            addend = SAs(j - 1) if SQ_KFOLD else "0"
        else:
            addend = "0" if j == NW else SAs(j)
        out.append(f"v_mad_u64_u32 {SAs(j - 1)}, vcc, {SX0D}, {SB1(j)}, {addend}")
        if j == 2:
            out.append(f"v_and_b32 {SQ}, {MASK}, {SQ}")
        if j == 4 and not SQ_KFOLD:
            out.append(f"v_sub_u32 {SCQ}, {kreg}, {SQ}")
        if j == 12:
            out.append(f"v_mad_i64_i32 {STS}, vcc, {SQ}, -1, {STS}" if SQ_KFOLD else
                       f"v_mad_u64_u32 {STS}, vcc, {SCQ}, 1, {STS}")
        if j == 20:
            out.append(f"v_mul_lo_u32 {SQ2}, {STSLO}, {SNPV}")
        if j == 26:
            out.append(f"v_and_b32 {SQ2}, {MASK}, {SQ2}")
    # ---- t part: doubled cross products 2 x0_i x0_k, k > i (the top position written fresh) ----
    for k in range(i + 1, L):
        addend = "0" if (first or k == L - 1) else SAt(k)
        out.append(f"v_mad_u64_u32 {SAt(k)}, vcc, {SX0D}, {SB0(k)}, {addend}")
    # ---- t: q * N (shifting the window);  s: q' * N ----
    top = "0" if last else SAt(L - 1)
    out.append(f"v_mad_u64_u32 {STT}, vcc, {SQ}, {Ns(0)}, {SAt(0)}")
    for k in range(1, L):
        out.append(f"v_mad_u64_u32 {SAt(k - 1)}, vcc, {SQ}, {Ns(k)}, {SAt(k) if k < L - 1 else top}")
    out.append(f"v_mad_u64_u32 {STS}, vcc, {SQ2}, {Ns(0)}, {STS}")
    for j in range(1, L):
        out.append(f"v_mad_u64_u32 {SAs(j - 1)}, vcc, {SQ2}, {Ns(j)}, {SAs(j - 1)}")
    out += [f"v_lshrrev_b64 {STT}, {LB}, {STT}", f"v_lshl_add_u64 {SAt(0)}, {STT}, 0, {SAt(0)}",
            f"v_lshrrev_b64 {STS}, {LB}, {STS}", f"v_lshl_add_u64 {SAs(0)}, {STS}, 0, {SAs(0)}"]
    if not last:
        out += ["s_waitcnt lgkmcnt(0)", f"v_lshlrev_b32 {SX0D}, 1, {SX0N}"]
    return out


def square_unrolled():
    body = list(load_consts())
    body.append(f"v_add_u32 {STMP}, 0x10000, %[a]")
    for j in range(2 * L):
        reg = SB0(j) if j < L else SB1(j - L)
        if j < 64:
            body.append(f"ds_read_b32 {reg}, %[a] offset:{j * 1024}")
        else:
            body.append(f"ds_read_b32 {reg}, {STMP} offset:{(j - 64) * 1024}")
    if SQ_KFOLD:  # the s window starts at the pairs (K'_j, 0): column j's K'_j, added once
        body += [f"ds_read_b64 {STS}, %[k]"] + [f"ds_read_b64 {SAs(j - 1)}, %[k] offset:{8 * j}" for j in range(1, L)]
    body += [f"v_mov_b32 {SNPV}, %[np]", f"ds_read_b32 {SX0}, %[a]", "s_waitcnt lgkmcnt(0)",
             f"v_lshlrev_b32 {SX0D}, 1, {SX0}"]
    for i in range(L):
        body += sq_row_static(i)
        # the mid-product reduction: the t part after row SQ_MID_T - 1, the s part after row SQ_MID_S - 1
        # (interleaved when both fall after the same row), each on its SQ_MID_KEEP slots
        t_regs, s_regs = [SAtLo(k) for k in range(L - 1)], [SAsLo(k) for k in range(NW)]
        keep = SQ_MID_KEEP or (None, None)
        parts = ([t_regs], [keep[0]]) if i == SQ_MID_T - 1 else ([], [])
        if i == SQ_MID_S - 1:
            parts = (parts[0] + [s_regs], parts[1] + [keep[1]])
        if parts[0]:
            one = [set() if r is t_regs else sq_one_slots() for r in parts[0]] if SQ_KFOLD else None
            body += mid_reduce(parts[0], keep=None if SQ_MID_KEEP is None else parts[1], one=one)
    # diagonals of columns L .. 2L-2 (h >= L/2): column 2h sits at window position 2h - L
    body += [f"v_mad_u64_u32 {SAt(2 * h - L)}, vcc, {SB0(h)}, {SB0(h)}, {SAt(2 * h - L)}" for h in range(L // 2, L)]
    body.append(f"v_add_u32 {STMP}, 0x10000, %[a]")

    def st(k, reg):
        if k < 64:
            return f"ds_write_b32 %[a], {reg} offset:{k * 1024}"
        return f"ds_write_b32 {STMP}, {reg} offset:{(k - 64) * 1024}"

    for acc, lo, carry, carry_lo, base in ((SAt, SAtLo, STT, STTLO, 0), (SAs, SAsLo, STS, STSLO, L)):
        body += [f"v_lshrrev_b64 {carry}, {LB}, {acc(0)}", f"v_and_b32 {lo(0)}, {MASK}, {lo(0)}", st(base, lo(0))]
        for k in range(1, NW):
            body += [f"v_lshl_add_u64 {acc(k)}, {carry}, 0, {acc(k)}",
                     f"v_lshrrev_b64 {carry}, {LB}, {acc(k)}",
                     f"v_and_b32 {lo(k)}, {MASK}, {lo(k)}",
                     st(base + k, lo(k))]
        body.append(st(base + NW, carry_lo))
    body.append("s_waitcnt lgkmcnt(0)")
    return rotate_carries(body)


def sq_mads():
    """64-bit multiply-adds per square: triangular t part (cross products + diagonals), the s part's
    (2 x0) x1 and - q (K' - q), the two q N passes, the mid-product reduction (its kept slots)."""
    if UNROLLED_SQUARE:
        return count_mads(square_unrolled())
    cross = L * (L - 1) // 2
    return cross + L + L * L + (L * L + L + L * L) + (L - 2) + (NW - 1)


def mm_mads():
    return L * (5 * L + 1) + 2 * (NW - 1)


def clobbers():
    regs = [f'"v{i}"' for i in range(max(MM_NREG, SQ_NREG, MS_NREG))]
    regs += [f'"s{i}"' for i in [16, 17] + list(range(19, 32)) + [34, 35] + list(range(36, 100))]
    out = [", ".join(regs[i:i + 16]) for i in range(0, len(regs), 16)]
    return " \\\n  ".join(x + "," for x in out[:-1]) + " \\\n  " + out[-1]


def c_string(lines):
    return "\n".join(f'  "{ln}\\n"' for ln in lines)


def count_mads(lines):
    return sum(1 for ln in lines if ln.startswith(("v_mad_u64_u32", "v_mad_i64_i32")))


def main():
    mm, sq, ms = product(False), (square_unrolled() if UNROLLED_SQUARE else square_tri()), mul_short_reg()
    sq_looped = square_tri()
    mm_row, sq_body = row(False, False), sq_row("odd")
    hdr = f"""// GENERATED by tools/gen_nadic_asm.py -- do not edit by hand.
//
// gfx950 assembly Montgomery product modulo N^2 in N-adic form: a residue is two {L}-limb
// digits (x0, x1), X = x0 + x1 N (mod N^2), radix 2^{LB}, R = 2^{LB * L}.
//   a (per-lane LDS column, {2 * L} limbs) <- a * b * R^-1 (mod N^2), digits lazily < 2N.
// See tools/gen_nadic_asm.py for the arithmetic, the bounds and the register plan.
// {len(mm)} instructions (general, B from global), {len(sq)} (square, triangular x0^2); row
// bodies {len(mm_row)} / <= {len(sq_body)} instructions; {mm_mads()} / {sq_mads()} v_mad_u64_u32 per product;
// the short-base product (h < 2^{LB * KS}, {KS} rows): {len(ms)} instructions, {ms_mads()} v_mad_u64_u32.
#pragma once
#include <stdint.h>

#define FBM_NA_LIMB_BITS {LB}
#define FBM_NA_LIMBS {L}
#define FBM_NA_MADS_MUL {mm_mads()}
#define FBM_NA_MADS_SQR {sq_mads()}
#define FBM_NA_MADS_SHORT {ms_mads()}
#define FBM_NA_SHORT_LIMBS {KS}
// the square's s window starts at the pairs (2^29 - 1 + P'_j, 0), P' = (K - E) mod N, K = (1 - R) mod N,
// E = sum of 2^(32 + 29 c) over the columns c set in this mask (the mid-product reduction leaves them at
// 2^32 + low dword: sq_kfold_extra in the generator).  The short product's: (D'_j, 0) (mul_short_reg).
#define FBM_NA_SQ_ONE_MASK {hex(sum(1 << (SQ_MID_S + k) for k in sq_one_slots()) if SQ_KFOLD else 0)}ull

#define FBM_NA_CLOBBERS \\
  {clobbers()}

// B operand from global memory: limb k at bb + b_off + k*1024 (bytes; bb uniform).
// NK: the 80-word constants block (N limbs, K'_i); np = -N^-1 mod 2^{LB}.
__device__ __forceinline__ void fbm_na_mm_glb(uint32_t a_off, const uint32_t* bb, uint32_t b_off,
                                              const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(mm)}
      :
      : [a] "v"(a_off), [b] "v"(b_off), [bb] "s"(bb), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}

// a <- a * (1, p) R^-1 (mod N^2): the encrypt's nude = N p + 1, digit 1's limb k at bb + b_off + k*1024
// (digit 0 = 1 as immediates: jl_nude_kernel stores only digit 1)
__device__ __forceinline__ void fbm_na_mm_nude(uint32_t a_off, const uint32_t* bb, uint32_t b_off,
                                               const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(product(False, nude=True))}
      :
      : [a] "v"(a_off), [b] "v"(b_off), [bb] "s"(bb), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}

// a <- a * h * 2^-{LB * KS} (mod N^2) for a short h = (h, 0), h < 2^{LB * KS}: h's {KS} limbs in registers,
// d: LDS byte address of the pairs (D'_j, 0), D'_j = D_j + (2^29 - 1) [j < {KS}] + [j == 0], D = N - 2^{LB * KS}
// (36 x 8 bytes).
__device__ __forceinline__ void fbm_na_ms_reg(uint32_t a_off, const uint32_t (&h)[{KS}], uint32_t d_off,
                                              const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(ms)}
      :
      : [a] "v"(a_off), {", ".join(f'[h{i}] "v"(h[{i}])' for i in range(KS))}, [d] "v"(d_off), [NK] "s"(NK),
        [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}

#if !defined(FBM_NA_PLAIN_SQUARE) && !defined(FBM_NA_LOOPED_SQUARE)
// a <- a^2 R^-1 (mod N^2): triangular x0^2, full x0 * 2 x1, every row unrolled ({len(sq)} instructions);
// k: LDS byte address of the s window's initial pairs (2^29 - 1 + P'_j, 0) (FBM_NA_SQ_ONE_MASK).
__device__ __forceinline__ void fbm_na_sq_lds(uint32_t a_off, uint32_t k_off, const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(sq)}
      :
      : [a] "v"(a_off), [k] "v"(k_off), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}
#elif defined(FBM_NA_LOOPED_SQUARE)
// A/B variant (-DFBM_NA_LOOPED_SQUARE): the row loop with computed-jump row suffixes ({len(sq_looped)} instructions).
__device__ __forceinline__ void fbm_na_sq_lds(uint32_t a_off, uint32_t, const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(sq_looped)}
      :
      : [a] "v"(a_off), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}
#else
// A/B variant (-DFBM_NA_PLAIN_SQUARE): the general product with B = A from LDS -- no computed
// jumps, {L * count_mads(row(False, True)) + 2 * (NW - 1)} multiplies instead of {sq_mads()}.
__device__ __forceinline__ void fbm_na_sq_lds(uint32_t a_off, uint32_t, const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(product(True))}
      :
      : [a] "v"(a_off), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}
#endif

// The looped triangular square (computed-jump row suffixes, {len(sq_looped)} instructions): the table path's squares
// (small moduli, FDH retries -- cold), so the launch's hot code keeps one copy of the unrolled square.
__device__ __forceinline__ void fbm_na_sq_lds_looped(uint32_t a_off, const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(sq_looped)}
      :
      : [a] "v"(a_off), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}: general {len(mm)} / square {len(sq)} instructions; "
          f"mads/product {mm_mads()} / {sq_mads()}")


if __name__ == "__main__":
    main()
