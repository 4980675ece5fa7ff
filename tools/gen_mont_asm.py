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
a_off squares) or from global memory (uniform base + per-lane byte offset, limb stride
1024 B: the workgroup-blocked [limb][lane] layout of the tables and residue columns).
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
    body += load_b_lds() if bsrc == "lds" else load_b_global()
    body += [f"v_mov_b32 {MPV}, %[mp]", f"v_mov_b32 {AADR}, %[a]", f"ds_read_b32 {AI}, {AADR}"]
    body += ["s_waitcnt vmcnt(0) lgkmcnt(0)"]
    body += row(True)
    body += ["s_mov_b32 s34, 1", "1:"]
    body += row(False)
    body += ["s_add_u32 s34, s34, 1", f"s_cmp_lg_u32 s34, {NL}", "s_cbranch_scc1 1b"]
    body += normalise_store()
    return body


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
    lds, glb = product("lds"), product("global")
    hdr = f"""// GENERATED by tools/gen_mont_asm.py -- do not edit by hand.
//
// gfx950 assembly Montgomery product, radix 2^28, 74 limbs (modulus N^2 <= 2048 bits,
// R = 2^2072).  a (per-lane LDS column) <- a * b * R^-1, lazily reduced (< 2M for a, b < 2M).
// See tools/gen_mont_asm.py for the register plan and the arithmetic; fbm_mont.hpp's
// mont_mul<74> is the same computation in C++.
// {len(lds)} instructions (B from LDS), {len(glb)} (B from global); the row loop body is {len(row(False))}.
#pragma once
#include <stdint.h>

#define FBM_MM_CLOBBERS \\
  {clobbers()}

// B operand from an LDS column: b_off = LDS byte address of b_0 (limb stride 1024 B).
// b_off == a_off computes a square.
__device__ __forceinline__ void fbm_mm_lds(uint32_t a_off, uint32_t b_off, const uint32_t* M, uint32_t mp) {{
  asm volatile(
{c_string(lds)}
      :
      : [a] "v"(a_off), [b] "v"(b_off), [M] "s"(M), [mp] "s"(mp)
      : "memory", "vcc", "scc", FBM_MM_CLOBBERS);
}}

// B operand from global memory: limb k at bb + b_off + k*1024 (bytes; bb uniform).
__device__ __forceinline__ void fbm_mm_glb(uint32_t a_off, const uint32_t* bb, uint32_t b_off, const uint32_t* M,
                                           uint32_t mp) {{
  asm volatile(
{c_string(glb)}
      :
      : [a] "v"(a_off), [b] "v"(b_off), [bb] "s"(bb), [M] "s"(M), [mp] "s"(mp)
      : "memory", "vcc", "scc", FBM_MM_CLOBBERS);
}}
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}: lds {len(lds)} / global {len(glb)} instructions")


if __name__ == "__main__":
    main()
