#!/usr/bin/env python3
"""Generate fedbiomed_amd/csrc/fbm_mont_asm.hpp: the gfx950 assembly Montgomery product.

Why assembly: the radix-2^28 product keeps 73 64-bit column accumulators that shift by one
column per row.  In C++ the row loop has to be fully unrolled (LLVM cannot coalesce the
loop-carried shift), giving ~90 KB of straight-line code per product -- far larger than the
instruction cache, so every wave streams its instructions from L2 (measured: ~40 cycles per
VALU instruction instead of ~4.5).  Written directly against fixed registers the shift is
just the choice of destination register (A[j-1] <- A[j] + ...), so the 74 rows run as a
runtime loop over one ~1.2 KB body and the whole product stays I-cache resident.

Register plan (per lane, wave64):
  v[2k:2k+1]  k=0..72   column accumulators A_k (64-bit)
  v146..v219            B operand limbs b_0..b_73 (28-bit)
  v220, v221            a_i (current row), a_{i+1} (prefetched from LDS)
  v[222:223]            T = A_0 + a_i*b_0 + m*M_0 (retired column)
  v224                  m = T * mp mod 2^28
  v225                  mp
  v[226:227]            carry
  v228, v229            running LDS address of a_i / scratch address
  s36..s99, s20..s29    modulus limbs M_0..M_63, M_64..M_73 (uniform, loaded once)
  s34                   row counter;  vcc: the (unused) carry-out of v_mad_u64_u32;
                        scc: the row-loop compare (declared clobbered: the compiler
                        would otherwise keep a branch condition in it across the asm)
s32/s33 (ABI stack/frame) and s100/s101 (reserved on gfx950) are left alone.

Arithmetic (identical to mont_mul in fbm_mont.hpp, which is the C++ statement of it):
  for i in 0..73:  T = A_0 + a_i b_0;  m = (T mp) & (2^28-1);  T += m M_0
                   A_{j-1} = A_j + a_i b_j + m M_j   (j = 1..72);   A_72 = a_i b_73 + m M_73
                   A_0 += T >> 28
  then normalise the columns to 74 limbs of 28 bits and store them to the A column in LDS.
Every column receives at most 148 products < 2^56 plus carries < 2^37: no 64-bit overflow.
Result < 2M whenever a, b < 2M (R = 2^2072 >= 4M): lazy reduction, as in fbm_mont.hpp.

Operands: the A operand is the lane's LDS column (limb k at byte a_off + k*1024) and is
overwritten by the result; B comes either from an LDS column (b_off, same stride; b_off ==
a_off squares) or (round 6) from the lane's 64-word little-endian row in global memory, converted
to 28-bit limbs in B's registers (fbm_mm_row: the combine kernels read their ciphertexts this way).
The LDS column must be allocated with 75 limb rows: the last row's a_{i+1} prefetch reads
row 74 (value unused).

Usage:  python tools/gen_mont_asm.py   (rewrites the header; the build does not run this)
"""

import os

NL = 74
NA = NL - 1  # 73 accumulators
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "fedbiomed_amd", "csrc", "fbm_mont_asm.hpp")

MASK = "0xfffffff"


def A(k):
    return f"v[{2 * k}:{2 * k + 1}]"


def Alo(k):
    return f"v{2 * k}"


def B(j):
    return f"v{146 + j}"


def Ms(j):
    return f"s{36 + j}" if j < 64 else f"s{20 + j - 64}"


AI, AN, T, TLO, MV, MPV, C, CLO, AADR, TMP = "v220", "v221", "v[222:223]", "v222", "v224", "v225", "v[226:227]", "v226", "v228", "v229"


def load_modulus():
    return [
        "s_load_dwordx16 s[36:51], %[M], 0x0",
        "s_load_dwordx16 s[52:67], %[M], 0x40",
        "s_load_dwordx16 s[68:83], %[M], 0x80",
        "s_load_dwordx16 s[84:99], %[M], 0xc0",
        "s_load_dwordx8 s[20:27], %[M], 0x100",
        "s_load_dwordx2 s[28:29], %[M], 0x120",
    ]


def load_b_lds():
    out = [f"v_add_u32 {TMP}, 0x10000, %[b]"]
    for j in range(NL):
        if j < 64:
            out.append(f"ds_read_b32 {B(j)}, %[b] offset:{j * 1024}")
        else:
            out.append(f"ds_read_b32 {B(j)}, {TMP} offset:{(j - 64) * 1024}")
    return out


def load_b_global():
    # the caller may just have stored this column (same lane): drain stores before loading
    out = ["s_waitcnt vmcnt(0)", f"v_mov_b32 {TMP}, %[b]"]
    for j in range(NL):
        if j and j % 4 == 0:
            out.append(f"v_add_u32 {TMP}, 0x1000, {TMP}")
        out.append(f"global_load_dword {B(j)}, {TMP}, %[bb] offset:{(j % 4) * 1024}")
    return out


def load_b_row():
    """B from the lane's own 2048-bit value as 64 little-endian 32-bit words at the per-lane byte address
    %[r] (a VGPR pair): a ciphertext row where the kernel's input already holds it -- no LDS staging
    column (round 6: the products then need 300 bytes of LDS per lane, not 600, and run two waves per
    SIMD).  Sixteen 16-byte loads into B's registers, then the 28-bit limbs in place, the top limb first
    (limb k reads words floor(28 k / 32) and the next, both at or below register k, and no limb above k
    reads those once it is written).  Issued with the A column's first read; converted after the wait."""
    return [f"global_load_dwordx4 v[{146 + 4 * i}:{149 + 4 * i}], %[r], off offset:{16 * i}" for i in range(16)]


def convert_b_row():
    out = []
    for k in range(NL - 1, -1, -1):
        w, sh = divmod(28 * k, 32)
        if sh + 28 <= 32 or w + 1 >= 64:  # inside word w (the top limb: its last 4 bits)
            out.append(f"v_bfe_u32 {B(k)}, {B(w)}, {sh}, {min(28, 32 - sh)}")
        else:  # straddles words w, w + 1
            out.append(f"v_alignbit_b32 {B(k)}, {B(w + 1)}, {B(w)}, {sh}")
            out.append(f"v_and_b32 {B(k)}, {MASK}, {B(k)}")
    return out


def row(first):
    """One row of the product; `first` = accumulators not yet initialised (addend 0)."""
    add = (lambda k: "0") if first else A
    out = [f"ds_read_b32 {AN}, {AADR} offset:1024"]
    out.append(f"v_mad_u64_u32 {T}, vcc, {AI}, {B(0)}, {add(0)}")
    for j in range(1, NL):
        addend = add(j) if j < NA else "0"
        out.append(f"v_mad_u64_u32 {A(j - 1)}, vcc, {AI}, {B(j)}, {addend}")
        if j == 3:
            out.append(f"v_mul_lo_u32 {MV}, {TLO}, {MPV}")
        if j == 6:
            out.append(f"v_and_b32 {MV}, {MASK}, {MV}")
    out.append(f"v_mad_u64_u32 {T}, vcc, {MV}, {Ms(0)}, {T}")
    for j in range(1, NL):
        out.append(f"v_mad_u64_u32 {A(j - 1)}, vcc, {MV}, {Ms(j)}, {A(j - 1)}")
    out.append(f"v_lshrrev_b64 {C}, 28, {T}")
    out.append(f"v_lshl_add_u64 {A(0)}, {C}, 0, {A(0)}")
    out.append(f"v_add_u32 {AADR}, 0x400, {AADR}")
    out.append("s_waitcnt lgkmcnt(0)")
    out.append(f"v_mov_b32 {AI}, {AN}")
    return out


def normalise_store():
    out = [f"v_add_u32 {TMP}, 0x10000, %[a]"]

    def st(k, reg):
        if k < 64:
            return f"ds_write_b32 %[a], {reg} offset:{k * 1024}"
        return f"ds_write_b32 {TMP}, {reg} offset:{(k - 64) * 1024}"

    out.append(f"v_lshrrev_b64 {C}, 28, {A(0)}")
    out.append(f"v_and_b32 {Alo(0)}, {MASK}, {Alo(0)}")
    out.append(st(0, Alo(0)))
    for k in range(1, NA):
        out.append(f"v_lshl_add_u64 {A(k)}, {C}, 0, {A(k)}")
        out.append(f"v_lshrrev_b64 {C}, 28, {A(k)}")
        out.append(f"v_and_b32 {Alo(k)}, {MASK}, {Alo(k)}")
        out.append(st(k, Alo(k)))
    out.append(st(NA, CLO))
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def product(bsrc):
    body = []
    body += load_modulus()
    body += {"lds": load_b_lds, "global": load_b_global, "row": load_b_row}[bsrc]()
    body += [f"v_mov_b32 {MPV}, %[mp]", f"v_mov_b32 {AADR}, %[a]", f"ds_read_b32 {AI}, {AADR}"]
    body += ["s_waitcnt vmcnt(0) lgkmcnt(0)"]
    if bsrc == "row":
        body += convert_b_row()
    body += row(True)
    body += ["s_mov_b32 s34, 1", "1:"]
    body += row(False)
    body += ["s_add_u32 s34, s34, 1", f"s_cmp_lg_u32 s34, {NL}", "s_cbranch_scc1 1b"]
    body += normalise_store()
    return body


# ------------------------------------------------------------------------------------------
# Squaring: a <- a^2 * R^-1.  Same result bit for bit as product("lds") with b == a, about
# 25 % fewer multiplies.  Row r adds only the doubled cross products 2 a_r a_k (k > r) --
# a contiguous suffix of the row's multiply sequence, entered by a computed jump
# (s_setpc_b64: every v_mad_u64_u32 is 8 bytes) -- plus the diagonal a_{r/2}^2 of column r
# (even r only, read from the LDS column along a running address: rows are unrolled in
# odd/even pairs so the parity is static).  Diagonals of columns 74..146 are added after the
# loop from the B registers.
# Every column holds the same total as in the general product when its m is computed, so
# the Montgomery quotients and the result are identical.  Column bound: <= 37 doubled
# products (< 2^57) + 1 diagonal + 74 m*M products (< 2^56) + carries < 2^63.3.
# The a*b pass is in place and the m*M pass shifts the window (A_{k-1} <- A_k + m M_k),
# so the accumulator window has 74 pairs (A_73 is written, not accumulated, by each row).
# Register plan: A_k v[2k:2k+1] (k=0..73), B_k = a_k v148..v221, a_r of even / odd rows
# (doubled in place) v222 / v223, T v[224:225], m v226, mp v227, LDS address v228, scratch
# v229, diagonal limb v230, its LDS address v231;  s[30:31] jump target, s34 row, s35 scratch.
# ------------------------------------------------------------------------------------------
SQ_A = lambda k: f"v[{2 * k}:{2 * k + 1}]"  # noqa: E731
SQ_ALO = lambda k: f"v{2 * k}"  # noqa: E731
SQ_B = lambda j: f"v{148 + j}"  # noqa: E731
SQ_AI = ("v222", "v223")  # a_r of even / odd rows (doubled in place)
SQ_T, SQ_TLO, SQ_MV, SQ_MPV, SQ_AADR, SQ_TMP, SQ_DI, SQ_DADDR = (
    "v[224:225]", "v224", "v226", "v227", "v228", "v229", "v230", "v231")


def sq_tri(tag, first=False):
    """Doubled cross products of one row: A_k += (2 a_r) b_k for k > r.  Entered at k = r+1 by
    the caller's computed jump (or whole, for row 0).  k = 73 writes instead of adding: the
    previous row's shift pass left A_73 holding a value already consumed."""
    ai = SQ_AI[0] if tag in ("0", "e") else SQ_AI[1]
    out = [f"v_mad_u64_u32 {SQ_A(k)}, vcc, {ai}, {SQ_B(k)}, {'0' if first else SQ_A(k)}" for k in range(1, NA)]
    out.append(f"v_mad_u64_u32 {SQ_A(NA)}, vcc, {ai}, {SQ_B(NA)}, 0")
    return out


def sq_jump(tag, entry_sgpr_expr):
    """s[30:31] <- address of tri-block entry (k = entry); entry index from s34."""
    return ["s_getpc_b64 s[30:31]",
            f".Lfbm_sq_pc{tag}_%=:"] + entry_sgpr_expr + [
            "s_add_u32 s30, s30, s35",
            "s_addc_u32 s31, s31, 0",
            f"s_add_u32 s30, s30, .Lfbm_sq_tri{tag}_%= - .Lfbm_sq_pc{tag}_%=",
            "s_addc_u32 s31, s31, 0",
            "s_setpc_b64 s[30:31]",
            f".Lfbm_sq_tri{tag}_%=:"]


def sq_reduce(last=False):
    """Montgomery quotient of column r and the shifting m*M pass, then carry into A_0."""
    out = [f"v_mad_u64_u32 {SQ_T}, vcc, {SQ_MV}, {Ms(0)}, {SQ_A(0)}"]
    out += [f"v_mad_u64_u32 {SQ_A(k - 1)}, vcc, {SQ_MV}, {Ms(k)}, {SQ_A(k)}" for k in range(1, NA)]
    out.append(f"v_mad_u64_u32 {SQ_A(NA - 1)}, vcc, {SQ_MV}, {Ms(NA)}, {'0' if last else SQ_A(NA)}")
    out += [f"v_lshrrev_b64 {SQ_T}, 28, {SQ_T}", f"v_lshl_add_u64 {SQ_A(0)}, {SQ_T}, 0, {SQ_A(0)}"]
    return out


def sq_quotient(ai):
    return [f"v_mul_lo_u32 {SQ_MV}, {SQ_ALO(0)}, {SQ_MPV}", f"v_lshlrev_b32 {ai}, 1, {ai}",
            f"v_and_b32 {SQ_MV}, {MASK}, {SQ_MV}"]


def square():
    """Rows: 0 (peeled, even), pairs (r odd, r+1 even) for r = 1, 3, ..., 71, 73 (peeled, odd:
    no cross products left).  Even rows add the diagonal a_{r/2}^2 (prefetched from LDS along a
    running address); odd rows have none.  AADR = address of a_{r-1} at the top of a pair."""
    body = load_modulus()
    body.append(f"v_add_u32 {SQ_TMP}, 0x10000, %[a]")
    for j in range(NL):
        if j < 64:
            body.append(f"ds_read_b32 {SQ_B(j)}, %[a] offset:{j * 1024}")
        else:
            body.append(f"ds_read_b32 {SQ_B(j)}, {SQ_TMP} offset:{(j - 64) * 1024}")
    body += [f"v_mov_b32 {SQ_MPV}, %[mp]", f"v_mov_b32 {SQ_AADR}, %[a]", f"ds_read_b32 {SQ_AI[0]}, %[a]",
             f"ds_read_b32 {SQ_DI}, %[a]", f"v_add_u32 {SQ_DADDR}, 0x400, %[a]", "s_waitcnt lgkmcnt(0)"]
    # ---- row 0 (even; diagonal a_0^2; all cross products) ----
    body += [f"ds_read_b32 {SQ_AI[1]}, {SQ_AADR} offset:1024",
             f"v_mad_u64_u32 {SQ_A(0)}, vcc, {SQ_DI}, {SQ_DI}, 0",
             f"ds_read_b32 {SQ_DI}, {SQ_DADDR}"]  # diagonal of row 2: a_1
    body += sq_quotient(SQ_AI[0]) + sq_tri("0", first=True) + sq_reduce()
    body += ["s_waitcnt lgkmcnt(0)", "s_mov_b32 s34, 1", "1:"]
    # ---- odd row r (a_r in AI[1]; entry k = r+1 -> index r) ----
    body += [f"ds_read_b32 {SQ_AI[0]}, {SQ_AADR} offset:2048"]
    body += sq_quotient(SQ_AI[1])
    body += sq_jump("o", ["s_lshl_b32 s35, s34, 3"]) + sq_tri("o") + sq_reduce()
    body += ["s_waitcnt lgkmcnt(0)"]
    # ---- even row r+1 (a_{r+1} in AI[0]; diagonal a_{(r+1)/2}; entry index r+1) ----
    body += [f"ds_read_b32 {SQ_AI[1]}, {SQ_AADR} offset:3072",
             f"v_mad_u64_u32 {SQ_A(0)}, vcc, {SQ_DI}, {SQ_DI}, {SQ_A(0)}",
             f"v_add_u32 {SQ_DADDR}, 0x400, {SQ_DADDR}"]
    body += sq_quotient(SQ_AI[0])
    body += [f"ds_read_b32 {SQ_DI}, {SQ_DADDR}"]  # diagonal of the next even row
    body += sq_jump("e", ["s_add_u32 s35, s34, 1", "s_lshl_b32 s35, s35, 3"]) + sq_tri("e") + sq_reduce()
    body += [f"v_add_u32 {SQ_AADR}, 0x800, {SQ_AADR}", "s_waitcnt lgkmcnt(0)",
             "s_add_u32 s34, s34, 2", f"s_cmp_lg_u32 s34, {NL - 1}", "s_cbranch_scc1 1b"]
    # ---- row 73 (odd; no cross products; A_73 holds a consumed value -> addend 0) ----
    body += [f"v_mul_lo_u32 {SQ_MV}, {SQ_ALO(0)}, {SQ_MPV}", f"v_and_b32 {SQ_MV}, {MASK}, {SQ_MV}"]
    body += sq_reduce(last=True)
    # diagonals of columns 74..146 (column 2h lands at window position 2h - 74)
    body += [f"v_mad_u64_u32 {SQ_A(2 * h - NL)}, vcc, {SQ_B(h)}, {SQ_B(h)}, {SQ_A(2 * h - NL)}"
             for h in range((NL + 1) // 2, NL)]
    # normalise positions 0..72 (+ carry limb) and store to the A column
    body.append(f"v_add_u32 {SQ_TMP}, 0x10000, %[a]")

    def st(k, reg):
        if k < 64:
            return f"ds_write_b32 %[a], {reg} offset:{k * 1024}"
        return f"ds_write_b32 {SQ_TMP}, {reg} offset:{(k - 64) * 1024}"

    body += [f"v_lshrrev_b64 {SQ_T}, 28, {SQ_A(0)}", f"v_and_b32 {SQ_ALO(0)}, {MASK}, {SQ_ALO(0)}", st(0, SQ_ALO(0))]
    for k in range(1, NA):
        body += [f"v_lshl_add_u64 {SQ_A(k)}, {SQ_T}, 0, {SQ_A(k)}",
                 f"v_lshrrev_b64 {SQ_T}, 28, {SQ_A(k)}",
                 f"v_and_b32 {SQ_ALO(k)}, {MASK}, {SQ_ALO(k)}",
                 st(k, SQ_ALO(k))]
    body += [st(NA, SQ_TLO), "s_waitcnt lgkmcnt(0)"]
    return body


def sq_row_len():
    return len(sq_tri("o")) + len(sq_reduce()) + 12


def sq_clobbers():
    regs = [f'"v{i}"' for i in range(232)]
    regs += [f'"s{i}"' for i in list(range(20, 32)) + [34, 35] + list(range(36, 100))]
    out = [", ".join(regs[i:i + 16]) for i in range(0, len(regs), 16)]
    return " \\\n  ".join(x + "," for x in out[:-1]) + " \\\n  " + out[-1]


def c_string(lines):
    return "\n".join(f'  "{ln}\\n"' for ln in lines)


def clobbers():
    regs = [f'"v{i}"' for i in range(230)]
    regs += [f'"s{i}"' for i in list(range(20, 30)) + [34] + list(range(36, 100))]
    out, line = [], []
    for r in regs:
        line.append(r)
        if len(line) == 16:
            out.append(", ".join(line))
            line = []
    if line:
        out.append(", ".join(line))
    return " \\\n  ".join(s + "," for s in out[:-1]) + " \\\n  " + out[-1]


def main():
    lds, rw, sq = product("lds"), product("row"), square()
    hdr = f"""// GENERATED by tools/gen_mont_asm.py -- do not edit by hand.
//
// gfx950 assembly Montgomery product, radix 2^28, 74 limbs (modulus N^2 <= 2048 bits,
// R = 2^2072).  a (per-lane LDS column) <- a * b * R^-1, lazily reduced (< 2M for a, b < 2M).
// See tools/gen_mont_asm.py for the register plan and the arithmetic; fbm_mont.hpp's
// mont_mul<74> is the same computation in C++.
// {len(lds)} instructions (B from LDS), {len(rw)} (B from a 64-word row), {len(sq)} (square); row loop
// bodies {len(row(False))} and ~{sq_row_len()} per square row (its a*b part is entered part-way).
#pragma once
#include <stdint.h>

#define FBM_MM_CLOBBERS \\
  {clobbers()}

#define FBM_SQ_CLOBBERS \\
  {sq_clobbers()}

// B operand from an LDS column: b_off = LDS byte address of b_0 (limb stride 1024 B).
// b_off == a_off computes a square.
__device__ __forceinline__ void fbm_mm_lds(uint32_t a_off, uint32_t b_off, const uint32_t* M, uint32_t mp) {{
  asm volatile(
{c_string(lds)}
      :
      : [a] "v"(a_off), [b] "v"(b_off), [M] "s"(M), [mp] "s"(mp)
      : "memory", "vcc", "scc", FBM_MM_CLOBBERS);
}}

// B operand from global memory: the lane's b < 2^2048 as 64 little-endian words at `row` (a ciphertext row as
// the kernels receive it; 16-byte aligned).  The caller's own stores to that row must be complete (the
// product does not wait for them).
__device__ __forceinline__ void fbm_mm_row(uint32_t a_off, const uint32_t* row, const uint32_t* M, uint32_t mp) {{
  asm volatile(
{c_string(rw)}
      :
      : [a] "v"(a_off), [r] "v"(row), [M] "s"(M), [mp] "s"(mp)
      : "memory", "vcc", "scc", FBM_MM_CLOBBERS);
}}

// a <- a^2 R^-1 (identical to fbm_mm_lds(a_off, a_off, ...), ~25 % fewer multiplies).
__device__ __forceinline__ void fbm_sq_lds(uint32_t a_off, const uint32_t* M, uint32_t mp) {{
  asm volatile(
{c_string(sq)}
      :
      : [a] "v"(a_off), [M] "s"(M), [mp] "s"(mp)
      : "memory", "vcc", "scc", FBM_SQ_CLOBBERS);
}}
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}: lds {len(lds)} / row {len(rw)} / square {len(sq)} instructions")


if __name__ == "__main__":
    main()
