#!/usr/bin/env python3
"""Generate fedbiomed_amd/csrc/fbm_nadic_asm.hpp: the gfx950 assembly Montgomery product
modulo N^2 in N-adic form (the Joye-Libert exponentiation engine).

Why N-adic: the JL modulus is N^2 with N known (1024-bit biprime).  A residue X mod N^2 is
carried as two 37-limb digits (x0, x1), X = x0 + x1 N (mod N^2), and since N^2 = 0 the
product needs no x1*y1 term:

    X Y = x0 y0 + N (x0 y1 + x1 y0)                      (mod N^2)

With R = 2^1036 (37 limbs of 28 bits) and one Montgomery reduction modulo N of x0 y0,
x0 y0 + m N = t R  (m = the reduction's quotient digits), we get N R^-1 = N (R^-1 mod N)
(mod N^2) and therefore

    X Y R^-1 = t + N * REDC_N(x0 y1 + x1 y0 - m)          (mod N^2)

i.e. the Montgomery product modulo N^2 is two interleaved Montgomery products modulo N
that share their row loop: the t part reduces x0*y0 and hands its quotient digit q_i of
row i straight to the s part, which adds (K'_i - q_i) in that row's retiring column.
-m is taken as (R - 1 - m) + K with K = (1 - R) mod N, so every column stays non-negative:
K'_i = (2^28 - 1) + K_i (host constants).  Per product 37 rows x (37 + 37 + 74 + 37)
= 6 845 v_mad_u64_u32 (square: x0*x0 and x0*(2 x1): 5 476) against 10 952 / 8 288 for
the 74-limb Montgomery product modulo N^2 (fbm_mont_asm.hpp) -- the same arithmetic
result class at 0.63x / 0.66x of the multiplies.

Bounds (N < 2^1024, R = 2^1036 >= 2^12 N): digits < 2N in -> digits < 2N out
(t < N + 4N^2/R, s < N + 1 + (8N^2 + N)/R).  A digit up to R - 1 in one operand (the
hash h < 2^1036 entering as (h, 0), the plaintext digit of N*pt + 1 = (1, pt)) gives
digits < 3N + 1, which the next product brings back below 2N.  Columns: at most
111 products < 2^56 plus carries: < 2^63.

Register plan (per lane, wave64):
  v[2k:2k+1]      k=0..35  t-window accumulators At_k (64-bit)
  v[72+2k:73+2k]  k=0..35  s-window accumulators As_k
  v144..v180      B digit 0 limbs b0_j   (square: x0)
  v181..v217      B digit 1 limbs b1_j   (square: 2 x1, 29-bit limbs)
  v218, v219      x0_i, x1_i of the current row;  v220, v221 the next row's (prefetch)
  v[222:223]      Tt = retiring column of the t part;  v[224:225] Ts (s part)
  v226 q, v227 q', v228 np = -N^-1 mod 2^28, v229 LDS address of x0_i, v230 scratch,
  v231 K'_i - q
  s20..s29, s36..s62   N_0..N_9, N_10..N_36 (uniform, loaded once per product)
  s63..s99             K'_0..K'_36 (row i reads K'_i by s_movrels with m0 = i)
  s34 row counter, s35 K'_i;  vcc: unused carry-out of v_mad_u64_u32;  scc clobbered;
  m0 (reserved to the compiler) saved in s19 on entry and restored on exit.

Operands: A is the lane's LDS column (limb k of the 74 at byte a_off + k*1024: rows 0..36
digit 0, rows 37..73 digit 1; 75 rows allocated, the last row's prefetch reads row 74)
and receives the result; B comes from global memory (uniform base + per-lane byte offset,
limb stride 1024 B: the workgroup-blocked layout of tables and residue columns) or, for
the square, from the A column itself.  The constants block (80 words, see
NadicCtx in fbm_internal.hpp) holds N_0..N_9 at words 0..9 and
N_10..N_36, K'_0..K'_36 at words 16..79.

Usage:  python tools/gen_nadic_asm.py   (rewrites the header; the build does not run this)
"""

import os

L = 37
NW = L - 1  # window accumulators per part
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "fedbiomed_amd", "csrc", "fbm_nadic_asm.hpp")
MASK = "0xfffffff"


def At(k):
    return f"v[{2 * k}:{2 * k + 1}]"


def AtLo(k):
    return f"v{2 * k}"


def As(k):
    return f"v[{72 + 2 * k}:{73 + 2 * k}]"


def AsLo(k):
    return f"v{72 + 2 * k}"


def B0(j):
    return f"v{144 + j}"


def B1(j):
    return f"v{181 + j}"


def Ns(j):
    return f"s{20 + j}" if j < 10 else f"s{36 + j - 10}"


KBASE = "s63"
X0, X1, X0N, X1N = "v218", "v219", "v220", "v221"
TT, TTLO, TS, TSLO = "v[222:223]", "v222", "v[224:225]", "v224"
Q, Q2, NPV, AADR, TMP, CQ = "v226", "v227", "v228", "v229", "v230", "v231"
ROW1 = 37 * 1024  # byte offset of digit 1 in the LDS column


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
            out.append(f"v_sub_u32 {CQ}, {kreg}, {Q}")  # K'_i - q_i  (>= 0: K'_i >= 2^28 - 1)
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
    out += [f"v_lshrrev_b64 {TT}, 28, {TT}", f"v_lshl_add_u64 {At(0)}, {TT}, 0, {At(0)}",
            f"v_lshrrev_b64 {TS}, 28, {TS}", f"v_lshl_add_u64 {As(0)}, {TS}, 0, {As(0)}",
            f"v_add_u32 {AADR}, 0x400, {AADR}", "s_waitcnt lgkmcnt(0)", f"v_mov_b32 {X0}, {X0N}"]
    if not sq:
        out.append(f"v_mov_b32 {X1}, {X1N}")
    return out


def normalise_store():
    out = [f"v_add_u32 {TMP}, 0x10000, %[a]"]

    def st(k, reg):
        if k < 64:
            return f"ds_write_b32 %[a], {reg} offset:{k * 1024}"
        return f"ds_write_b32 {TMP}, {reg} offset:{(k - 64) * 1024}"

    for acc, lo, carry, carry_lo, base in ((At, AtLo, TT, TTLO, 0), (As, AsLo, TS, TSLO, L)):
        out += [f"v_lshrrev_b64 {carry}, 28, {acc(0)}", f"v_and_b32 {lo(0)}, {MASK}, {lo(0)}", st(base, lo(0))]
        for k in range(1, NW):
            out += [f"v_lshl_add_u64 {acc(k)}, {carry}, 0, {acc(k)}",
                    f"v_lshrrev_b64 {carry}, 28, {acc(k)}",
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
        if ln.startswith("v_mad_u64_u32") and ", vcc," in ln:
            ln = ln.replace(", vcc,", f", {pairs[i % len(pairs)]},", 1)
            i += 1
        out.append(ln)
    return out


def product(sq):
    body = [f"s_mov_b32 {M0_SAVE}, m0"] + load_consts()
    body += load_b_square() if sq else load_b_global()
    body += [f"v_mov_b32 {NPV}, %[np]", f"v_mov_b32 {AADR}, %[a]", f"ds_read_b32 {X0}, {AADR}"]
    if not sq:
        body.append(f"ds_read_b32 {X1}, {AADR} offset:{ROW1}")
    body += ["s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body += row(True, sq)
    # s_movrels after an SALU write of m0 needs a wait state (the hazard is not checked in asm)
    body += ["s_mov_b32 s34, 1", "1:", "s_mov_b32 m0, s34", "s_nop 1", f"s_movrels_b32 s35, {KBASE}"]
    body += row(False, sq)
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
# rows are unrolled in odd/even pairs so the parity is static).  Diagonals of columns 38..72
# are added after the loop from the B registers.  The t products are added in place
# (At_k, k = window position) and the q*N pass shifts the window, so the t window has 37
# pairs (At_36 is written, not accumulated, by each row's last cross product).  Column i is
# complete when its quotient is taken: cross products of column i come from rows < i, the
# diagonal from row i itself.  The s part runs full rows of (2 x0_i) * x1 (the doubled row
# operand serves both parts).  Column bounds: t 18 doubled products < 2^57 + 1 diagonal +
# 37 q*N < 2^56; s 37 doubled products + 37 q'*N: < 2^63.
# Register plan: At_k v[2k:2k+1] (k=0..36), As_k v[74+2k:75+2k] (k=0..35), b0 = x0
# v146..v182, b1 = x1 v183..v219, x0_0 v220, next x0 v221, 2 x0_i v222, Tt v[224:225],
# Ts v[226:227], q v228, q' v229, np v230, LDS address v231, scratch v232, K'_i - q v233,
# diagonal limb v234, its LDS address v235;  s[30:31] jump target, s34 row, s35 K'_i / offset.
# ------------------------------------------------------------------------------------------
def SAt(k):
    return f"v[{2 * k}:{2 * k + 1}]"


def SAtLo(k):
    return f"v{2 * k}"


def SAs(k):
    return f"v[{74 + 2 * k}:{75 + 2 * k}]"


def SAsLo(k):
    return f"v{74 + 2 * k}"


def SB0(j):
    return f"v{146 + j}"


def SB1(j):
    return f"v{183 + j}"


SX0, SX0N, SX0D = "v220", "v221", "v222"
STT, STTLO, STS, STSLO = "v[224:225]", "v224", "v[226:227]", "v226"
SQ, SQ2, SNPV, SAADR, STMP, SCQ, SDI, SDADDR = "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235"


def sq_tri(tag, first=False):
    """Doubled cross products 2 x0_i x0_k, k = 1..36 (entered at k = i + 1 by the jump;
    whole, with addend 0, for row 0).  k = 36 writes: the shift consumed the old top."""
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
    """kind: 'first' (row 0), 'odd', 'even' (loop rows), 'r35' (odd, only k = 36 crosses),
    'last' (row 36, even, no crosses).  On entry X0 = x0_i; s35 = K'_i (kreg)."""
    first = kind == "first"
    even = kind in ("first", "even", "last")
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
    elif kind == "r35":
        out.append(f"v_mad_u64_u32 {SAt(L - 1)}, vcc, {SX0D}, {SB0(L - 1)}, 0")
    # ---- t: q * N (shifting the window);  s: q' * N ----
    top = "0" if kind == "last" else SAt(L - 1)
    out.append(f"v_mad_u64_u32 {STT}, vcc, {SQ}, {Ns(0)}, {SAt(0)}")
    for k in range(1, L):
        out.append(f"v_mad_u64_u32 {SAt(k - 1)}, vcc, {SQ}, {Ns(k)}, {SAt(k) if k < L - 1 else top}")
    out.append(f"v_mad_u64_u32 {STS}, vcc, {SQ2}, {Ns(0)}, {STS}")
    for j in range(1, L):
        out.append(f"v_mad_u64_u32 {SAs(j - 1)}, vcc, {SQ2}, {Ns(j)}, {SAs(j - 1)}")
    out += [f"v_lshrrev_b64 {STT}, 28, {STT}", f"v_lshl_add_u64 {SAt(0)}, {STT}, 0, {SAt(0)}",
            f"v_lshrrev_b64 {STS}, 28, {STS}", f"v_lshl_add_u64 {SAs(0)}, {STS}, 0, {SAs(0)}",
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
    body += sq_row("first", kreg=KBASE)
    body += ["s_mov_b32 s34, 1", "1:"]
    body += krow(["s_mov_b32 m0, s34"]) + sq_row("odd")
    body += krow(["s_add_u32 m0, s34, 1"]) + sq_row("even")
    body += ["s_add_u32 s34, s34, 2", f"s_cmp_lg_u32 s34, {L - 2}", "s_cbranch_scc1 1b"]
    body += krow(["s_mov_b32 m0, 35"]) + sq_row("r35")
    body += krow(["s_mov_b32 m0, 36"]) + sq_row("last")
    # diagonals of columns 38..72: column 2h sits at window position 2h - 37
    body += [f"v_mad_u64_u32 {SAt(2 * h - L)}, vcc, {SB0(h)}, {SB0(h)}, {SAt(2 * h - L)}" for h in range(19, L)]
    body.append(f"v_add_u32 {STMP}, 0x10000, %[a]")

    def st(k, reg):
        if k < 64:
            return f"ds_write_b32 %[a], {reg} offset:{k * 1024}"
        return f"ds_write_b32 {STMP}, {reg} offset:{(k - 64) * 1024}"

    for acc, lo, carry, carry_lo, base in ((SAt, SAtLo, STT, STTLO, 0), (SAs, SAsLo, STS, STSLO, L)):
        body += [f"v_lshrrev_b64 {carry}, 28, {acc(0)}", f"v_and_b32 {lo(0)}, {MASK}, {lo(0)}", st(base, lo(0))]
        for k in range(1, NW):
            body += [f"v_lshl_add_u64 {acc(k)}, {carry}, 0, {acc(k)}",
                     f"v_lshrrev_b64 {carry}, 28, {acc(k)}",
                     f"v_and_b32 {lo(k)}, {MASK}, {lo(k)}",
                     st(base + k, lo(k))]
        body.append(st(base + NW, carry_lo))
    body += ["s_waitcnt lgkmcnt(0)", f"s_mov_b32 m0, {M0_SAVE}", "s_nop 1"]
    return rotate_carries(body)


def sq_mads():
    """v_mad_u64_u32 per square (triangular t part)."""
    cross = L * (L - 1) // 2
    return cross + L + L * L + (L * L + L + L * L)


def clobbers():
    regs = [f'"v{i}"' for i in range(236)]
    regs += [f'"s{i}"' for i in [16, 17] + list(range(19, 32)) + [34, 35] + list(range(36, 100))]
    out = [", ".join(regs[i:i + 16]) for i in range(0, len(regs), 16)]
    return " \\\n  ".join(x + "," for x in out[:-1]) + " \\\n  " + out[-1]


def c_string(lines):
    return "\n".join(f'  "{ln}\\n"' for ln in lines)


def count_mads(lines):
    return sum(1 for ln in lines if ln.startswith("v_mad_u64_u32"))


def main():
    mm, sq = product(False), square_tri()
    mm_row, sq_body = row(False, False), sq_row("odd")
    hdr = f"""// GENERATED by tools/gen_nadic_asm.py -- do not edit by hand.
//
// gfx950 assembly Montgomery product modulo N^2 in N-adic form: a residue is two 37-limb
// digits (x0, x1), X = x0 + x1 N (mod N^2), radix 2^28, R = 2^1036.
//   a (per-lane LDS column, 74 limbs) <- a * b * R^-1 (mod N^2), digits lazily < 2N.
// See tools/gen_nadic_asm.py for the arithmetic, the bounds and the register plan.
// {len(mm)} instructions (general, B from global), {len(sq)} (square, triangular x0^2); row
// bodies {len(mm_row)} / <= {len(sq_body)} instructions; {L * count_mads(mm_row)} / {sq_mads()} v_mad_u64_u32 per product.
#pragma once
#include <stdint.h>

#define FBM_NA_MADS_MUL {L * count_mads(mm_row)}
#define FBM_NA_MADS_SQR {sq_mads()}

#define FBM_NA_CLOBBERS \\
  {clobbers()}

// B operand from global memory: limb k at bb + b_off + k*1024 (bytes; bb uniform).
// NK: the 80-word constants block (N limbs, K'_i); np = -N^-1 mod 2^28.
__device__ __forceinline__ void fbm_na_mm_glb(uint32_t a_off, const uint32_t* bb, uint32_t b_off,
                                              const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(mm)}
      :
      : [a] "v"(a_off), [b] "v"(b_off), [bb] "s"(bb), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}

#ifndef FBM_NA_PLAIN_SQUARE
// a <- a^2 R^-1 (mod N^2): triangular x0^2 (computed-jump row suffixes), full x0 * 2 x1.
__device__ __forceinline__ void fbm_na_sq_lds(uint32_t a_off, const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(sq)}
      :
      : [a] "v"(a_off), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}
#else
// A/B variant (-DFBM_NA_PLAIN_SQUARE): the general product with B = A from LDS -- no computed
// jumps, {L * count_mads(row(False, True))} multiplies instead of {sq_mads()}.
__device__ __forceinline__ void fbm_na_sq_lds(uint32_t a_off, const uint32_t* NK, uint32_t np) {{
  asm volatile(
{c_string(product(True))}
      :
      : [a] "v"(a_off), [NK] "s"(NK), [np] "s"(np)
      : "memory", "vcc", "scc", FBM_NA_CLOBBERS);
}}
#endif
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}: general {len(mm)} / square {len(sq)} instructions; "
          f"mads/product {L * count_mads(mm_row)} / {sq_mads()}")


if __name__ == "__main__":
    main()
