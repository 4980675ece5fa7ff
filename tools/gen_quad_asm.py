#!/usr/bin/env python3
"""Generate fedbiomed_amd/csrc/fbm_quad_asm.hpp: the N-adic Montgomery product modulo N^2
(tools/gen_nadic_asm.py has the arithmetic) spread over a QUAD of lanes -- four lanes per
ciphertext -- for launches with fewer ciphertexts than the chip has lanes.

Why: the one-lane engine's latency is one lane's whole exponentiation (~2 360 products), so a
launch holding fewer ciphertexts than resident lanes (the aggregate of a 1/8 stripe: 41 667
ciphertexts for 131 072 lanes) takes as long as a full one, with a third of the SIMDs idle.
Spread over four lanes, a ciphertext's product takes ~a quarter of the time and the 4x lanes
occupy every SIMD.  The price is more instructions per ciphertext (cross-lane steps, no
triangular square), so the library takes this engine only below ~7/16 of a one-lane round.

Radix: 29-bit limbs, 36 per digit (R = 2^1044 >= 2^20 N), 9 per lane -- 36 = 4 x 9 leaves no
padding slot (28-bit limbs would need 37, i.e. 10 slots per lane and 3 dead ones) and one row
fewer.  The price of 29 bits is the column bound: a row adds up to 3 products < 2^58 (x1 * b0,
x0 * b1, q' N; the square's doubled x1 makes 2^59 + 2^58), so 36 rows would overflow 64 bits;
after row 17 every slot hands its high dword to the slot above (x 8 = 2^32 / 2^29, one
v_mad_u64_u32) and keeps the low one, so each half of the rows starts from values < 2^36:
18 * 2^59.6 + 2^36 < 2^64.

Layout: lane l (= lane id mod 4) of the quad owns window slots and operand limbs 9 l .. 9 l + 8
of both digits.  Row i:
  * x0_i, x1_i (the row operand) are read from the ciphertext's LDS column by all four lanes
    (same address: an LDS broadcast), one row ahead, alternating between two register pairs
    (rows unrolled in pairs);
  * every lane adds x0_i * b0[r] (t part) and x0_i * b1[r] + x1_i * b0[r] (s part) for its 9
    limbs, the window shift done by register choice (the product of limb r goes to slot r - 1);
  * lane 0 holds column i: q = (T * (-N^-1)) mod 2^29 is masked and broadcast in one
    v_and_b32_dpp quad_perm [0,0,0,0]; every lane adds q * N[r]; the s part adds K'_i - q in
    lane 0 only (a multiply by e0 = [lane == 0]) and does the same with q';
  * retire: every lane splits its slot-0 value T = lo + c 2^29: c goes into its new slot 0,
    lo to the lane below as that lane's top slot (v_and_b32_dpp quad_perm [1,2,3,0]: mask and
    exchange in one instruction).  Exact for every lane: lo belongs one column lower than c.
    Lane 0's lo is the retiring column's, 0 after q N, and it rotates into lane 3's top slot,
    which must start the next row at 0 -- so the rotation needs no masking.
After the 36 rows each lane normalises its 9 slots (carry chain), passes its carry-out to the
lane above (quad_perm [3,0,1,2]; lane 3's is 0: results < 3N + 1 fit in 36 limbs) and folds it
into its slot 0 -- slot 1 may end one carry above 2^29 (a lazy limb, < 2^29 + 2^10).

The digits are the same residues the one-lane engine computes (with R = 2^1044 instead of
2^1036: Montgomery forms differ, canonical results are bit-identical); tests/test_quad_asm.py
interprets this assembly for whole quads against Python integers (and asserts every
v_mad_u64_u32 stays below 2^64), the -m gpu tests compare both engines and the oracle.

DPP hazards (the assembler inserts none): a VALU write of a VGPR followed by a DPP read of it
needs 2 wait states -- the Emitter checks every DPP against the preceding instructions and
pads with s_nop where the schedule does not already provide them.

Register plan (per lane):
  v[0:15]    At_0..At_7 (t window slots 0..7)     v[16:17] Tt (slot-0 result of the row)
  v[18:19]   Rt: slot 8 of t (v18 received, v19 = 0 except right after the mid-row reduction)
  v[20:35]   As_0..As_7                            v[36:37] Ts        v[38:39] Rs
  v40..v48   b0[0..8]      v49..v57 b1[0..8]
  v58, v59   x0, x1 of even rows    v60, v61 of odd rows
  v62 q  v63 q'  v64 K'_i - q  v65 LDS row address  v66 v67 scratch  v68 = 2^29 - 1
  v[70:71], v[72:73]  carry pairs (normalisation)  v74 v75 scratch
  s35, s36   K'_i of the pair's two rows (s_movrels from s64..s99), s34 row, s19 m0 save
  operands:  %[n0]..%[n8] the lane's N limbs (VGPRs the compiler keeps across products),
             %[e0] = [lane == 0], %[ac] the ciphertext column's LDS byte address (limb 0 of
             digit 0), %[al] = %[ac] + 9 l * ROW (the lane's slice), %[np] = -N^-1 mod 2^29
             (SGPR), %[QK] the quad constants block (K'_i at words 0..35).
LDS column: limb k of digit d at byte ac + (36 d + k) * ROW, ROW = 72 words * 4 (64 ciphertexts
per workgroup + 8 words of padding: the slice writes of a 32-lane half hit 32 distinct banks).

Usage:  python tools/gen_quad_asm.py   (rewrites the header; the build does not run this)
"""

import os

LB = 29         # bits per limb
L = 36          # limbs per digit
M = 9           # limbs per lane
ROWW = 72       # LDS words between limb rows
ROWB = ROWW * 4
D1 = L          # limb index of digit 1 in the LDS column
MID = 18        # rows before the mid-product reduction
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "fedbiomed_amd", "csrc", "fbm_quad_asm.hpp")
MASK = hex((1 << LB) - 1)


def At(k):
    return f"v[{2 * k}:{2 * k + 1}]"


def AtLo(k):
    return f"v{2 * k}"


def AtHi(k):
    return f"v{2 * k + 1}"


def As(k):
    return f"v[{20 + 2 * k}:{21 + 2 * k}]"


def AsLo(k):
    return f"v{20 + 2 * k}"


def AsHi(k):
    return f"v{21 + 2 * k}"


TT, TTLO = "v[16:17]", "v16"
RT, RTLO, RTHI = "v[18:19]", "v18", "v19"
TS, TSLO = "v[36:37]", "v36"
RS, RSLO, RSHI = "v[38:39]", "v38", "v39"


def B0(r):
    return f"v{40 + r}"


def B1(r):
    return f"v{49 + r}"


XA, XB = ("v58", "v59"), ("v60", "v61")
Q, Q2, CQ, AADR, TMP, TMP2, MASKV = "v62", "v63", "v64", "v65", "v66", "v67", "v68"
CY, CYLO, CYHI = "v[70:71]", "v70", "v71"
CS, CSLO, CSHI = "v[72:73]", "v72", "v73"
T3, T4 = "v74", "v75"
NREG = 76
KBASE = 64      # K'_i in s(64 + i)
M0_SAVE = "s19"


def N(r):
    return f"%[n{r}]"


def dpp(perm):
    return f"quad_perm:[{','.join(str(p) for p in perm)}] row_mask:0xf bank_mask:0xf"


class Emitter:
    """Collects instructions; pads with s_nop where a DPP reads a VGPR fewer than 2
    instructions after the VALU write of it (s_nop N counts N + 1 wait states)."""

    def __init__(self):
        self.out = []

    @staticmethod
    def dests(ln):
        op, _, rest = ln.partition(" ")
        if not op.startswith("v_") or not rest:
            return set()
        d = rest.split(",")[0].strip()
        if d.startswith("v["):
            lo, hi = d[2:-1].split(":")
            return {f"v{i}" for i in range(int(lo), int(hi) + 1)}
        return {d} if d.startswith("v") else set()

    def emit(self, ln):
        if "quad_perm" in ln:
            src = ln.split(",")[1].split()[0].strip()
            dist = 0
            for prev in reversed(self.out):
                if prev.endswith(":"):
                    break  # a label: assume the write is right before it
                if prev.startswith("s_nop"):
                    dist += int(prev.split()[1]) + 1
                elif prev.startswith("v_") and src in self.dests(prev):
                    break
                else:
                    dist += 1
                if dist >= 2:
                    break
            if dist < 2:
                self.out.append(f"s_nop {1 - dist}")
        self.out.append(ln)

    def extend(self, lines):
        for ln in lines:
            self.emit(ln)


def load_consts():
    # K'_0..K'_35 (words 0..35 of the quad constants block) -> s64..s99
    return ["s_load_dwordx16 s[64:79], %[QK], 0x0",
            "s_load_dwordx16 s[80:95], %[QK], 0x40",
            "s_load_dwordx4 s[96:99], %[QK], 0x80"]


def load_b_global():
    """b0[r] = limb row r, b1[r] = limb row 9 + r of the lane's quad-layout column: word
    (row * 256 + lane) of the 64-ciphertext block, rows 1 KB apart (%[b] = the lane's byte
    offset from the uniform %[bb])."""
    out = ["s_waitcnt vmcnt(0)", f"v_mov_b32 {TMP}, %[b]"]
    for j in range(2 * M):
        if j and j % 4 == 0:
            out.append(f"v_add_u32 {TMP}, 0x1000, {TMP}")
        reg = B0(j) if j < M else B1(j - M)
        out.append(f"global_load_dword {reg}, {TMP}, %[bb] offset:{(j % 4) * 1024}")
    return out


def load_b_lds(double_b1):
    out = []
    for r in range(M):
        out.append(f"ds_read_b32 {B0(r)}, %[al] offset:{r * ROWB}")
        out.append(f"ds_read_b32 {B1(r)}, %[al] offset:{(D1 + r) * ROWB}")
    out.append("s_waitcnt lgkmcnt(0)")
    if double_b1:  # square: the s part is x0 * (2 x1)
        out += [f"v_lshlrev_b32 {B1(r)}, 1, {B1(r)}" for r in range(M)]
    return out


def row(first, sq, kreg, xs, xn, pre_off):
    """One row with an explicit schedule (every dependent instruction 3+ instructions after
    its producer).  xs = this row's (x0, x1); xn = where the prefetch of the next row's
    operands goes, read at byte offset pre_off from AADR; kreg = K'_i."""
    x0, x1 = xs
    out = [f"ds_read_b32 {xn[0]}, {AADR} offset:{pre_off}"]
    if not sq:
        out.append(f"ds_read_b32 {xn[1]}, {AADR} offset:{pre_off + D1 * ROWB}")

    def addend(acc, r):
        if first:
            return "0"
        if r == M - 1:
            return RT if acc is At else RS
        return acc(r)

    def tm(r):  # t pass 1: x0 * b0[r]
        dst = TT if r == 0 else At(r - 1)
        return f"v_mad_u64_u32 {dst}, vcc, {x0}, {B0(r)}, {addend(At, r)}"

    def sm(r):  # s pass 1: x0 * b1[r]
        dst = TS if r == 0 else As(r - 1)
        return f"v_mad_u64_u32 {dst}, vcc, {x0}, {B1(r)}, {addend(As, r)}"

    # ---- pass 1: x0_i * b0 (t) and x0_i * b1 (s), the quotient chains threaded through ----
    p1 = [tm(0), sm(0), tm(1)]
    if not sq:
        p1.append(f"v_mad_u64_u32 {TS}, vcc, {x1}, {B0(0)}, {TS}")
    p1 += [tm(2), f"v_mul_lo_u32 {Q}, {TTLO}, %[np]", sm(1), tm(3), sm(2),
           f"v_and_b32_dpp {Q}, {Q}, {MASKV} {dpp((0, 0, 0, 0))}", sm(3), tm(4),
           f"v_sub_u32 {CQ}, {kreg}, {Q}", sm(4), tm(5),      # K'_i - q (>= 0: K'_i >= 2^29 - 1)
           f"v_mad_u64_u32 {TS}, vcc, {CQ}, %[e0], {TS}", sm(5), tm(6),
           f"v_mul_lo_u32 {Q2}, {TSLO}, %[np]", sm(6), tm(7), sm(7),
           f"v_and_b32_dpp {Q2}, {Q2}, {MASKV} {dpp((0, 0, 0, 0))}", tm(8), sm(8)]
    # ---- pass 2: q * N (t), interleaved with x1_i * b0 (s, general product) ----
    tq = [f"v_mad_u64_u32 {TT}, vcc, {Q}, {N(0)}, {TT}"] + \
        [f"v_mad_u64_u32 {At(r - 1)}, vcc, {Q}, {N(r)}, {At(r - 1)}" for r in range(1, M)]
    sx = [] if sq else [f"v_mad_u64_u32 {As(r - 1)}, vcc, {x1}, {B0(r)}, {As(r - 1)}" for r in range(1, M)]
    p2 = []
    for k in range(max(len(tq), len(sx))):
        if k < len(tq):
            p2.append(tq[k])
        if k < len(sx):
            p2.append(sx[k])
    # ---- pass 3: q' * N (s), both retires threaded in:
    #      T = lo + c 2^29 -> lo (masked) to the lane below's top slot, c into the new slot 0 ----
    sq3 = [f"v_mad_u64_u32 {TS}, vcc, {Q2}, {N(0)}, {TS}"] + \
        [f"v_mad_u64_u32 {As(r - 1)}, vcc, {Q2}, {N(r)}, {As(r - 1)}" for r in range(1, M)]
    ret_t = [f"v_and_b32_dpp {RTLO}, {TTLO}, {MASKV} {dpp((1, 2, 3, 0))}",
             f"v_lshrrev_b64 {TT}, {LB}, {TT}",
             f"v_lshl_add_u64 {At(0)}, {TT}, 0, {At(0)}"]
    ret_s = [f"v_and_b32_dpp {RSLO}, {TSLO}, {MASKV} {dpp((1, 2, 3, 0))}",
             f"v_lshrrev_b64 {TS}, {LB}, {TS}",
             f"v_lshl_add_u64 {As(0)}, {TS}, 0, {As(0)}"]
    p3 = [sq3[0], ret_t[0], sq3[1], ret_t[1], sq3[2], ret_t[2], sq3[3], ret_s[0], sq3[4], ret_s[1], sq3[5],
          ret_s[2]] + sq3[6:]
    return out + p1 + p2 + p3


def mid_reduce():
    """After row 17: every slot keeps its low dword and hands the high one to the slot above
    (x 8 = 2^32 / 2^29); the top slot's (R) high dword goes to the lane above's slot 0
    (lane 3's is 0: the window's value is below 2^1026).  Values drop below 2^36."""
    chains = []
    for acc, hi, rr, rhi, t in ((At, AtHi, RT, RTHI, T3), (As, AsHi, RS, RSHI, T4)):
        ch = []
        for k in range(M - 2):
            ch += [f"v_mad_u64_u32 {acc(k + 1)}, vcc, {hi(k)}, 8, {acc(k + 1)}", f"v_mov_b32 {hi(k)}, 0"]
        ch += [f"v_mad_u64_u32 {rr}, vcc, {hi(M - 2)}, 8, {rr}", f"v_mov_b32 {hi(M - 2)}, 0",
               f"v_mov_b32_dpp {t}, {rhi} {dpp((3, 0, 1, 2))}",
               f"v_mov_b32 {rhi}, 0",
               f"v_mad_u64_u32 {acc(0)}, vcc, {t}, 8, {acc(0)}"]
        chains.append(ch)
    out = []
    for a, b in zip(*chains):
        out += [a, b]
    return out


def normalise_store():
    """Window (slots 0..7 + R) -> 9 lazy 29-bit limbs per digit part, into the b registers
    (t -> b0, s -> b1), and the lane's slice of the LDS column.  The t and s carry chains are
    independent: interleaved instruction by instruction (a vcc add/addc pair kept together)."""
    chains = []
    for acc, lo, rr, rlo, breg, cy, cylo, cyhi, t1, t2 in (
            (At, AtLo, RT, RTLO, B0, CY, CYLO, CYHI, TMP, TMP2),
            (As, AsLo, RS, RSLO, B1, CS, CSLO, CSHI, T3, T4)):
        ch = [f"v_and_b32 {breg(0)}, {MASK}, {lo(0)}", f"v_lshrrev_b64 {cy}, {LB}, {acc(0)}"]
        for r in range(1, M - 1):
            ch += [f"v_lshl_add_u64 {acc(r)}, {cy}, 0, {acc(r)}",
                   f"v_and_b32 {breg(r)}, {MASK}, {lo(r)}",
                   f"v_lshrrev_b64 {cy}, {LB}, {acc(r)}"]
        ch += [f"v_lshl_add_u64 {rr}, {cy}, 0, {rr}",
               f"v_and_b32 {breg(M - 1)}, {MASK}, {rlo}",
               f"v_lshrrev_b64 {cy}, {LB}, {rr}",
               # carry-out -> the lane above (lane 0 receives lane 3's, which is 0)
               f"v_mov_b32_dpp {t1}, {cylo} {dpp((3, 0, 1, 2))}",
               f"v_mov_b32_dpp {t2}, {cyhi} {dpp((3, 0, 1, 2))}",
               f"v_add_co_u32 {t1}, vcc, {t1}, {breg(0)}|v_addc_co_u32 {t2}, vcc, 0, {t2}, vcc",
               f"v_and_b32 {breg(0)}, {MASK}, {t1}",
               f"v_alignbit_b32 {t1}, {t2}, {t1}, {LB}",  # (t2:t1) >> 29 (< 2^10: fits)
               f"v_add_u32 {breg(1)}, {breg(1)}, {t1}"]
        chains.append(ch)
    out = []
    for k in range(max(len(c) for c in chains)):
        for ch in chains:
            if k < len(ch):
                out += ch[k].split("|")
    for d, breg in ((0, B0), (1, B1)):
        out += [f"ds_write_b32 %[al], {breg(r)} offset:{(d * D1 + r) * ROWB}" for r in range(M)]
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def krow(dst, m0_expr):
    """dst <- K'_row (s_movrels after an SALU write of m0 needs a wait state)."""
    return [m0_expr, "s_nop 1", f"s_movrels_b32 {dst}, s{KBASE}"]


def pair(sq, first_x, second_x):
    """Rows (i, i+1) with i = s34; operands of row i in first_x, of row i+1 in second_x."""
    body = krow("s35", "s_mov_b32 m0, s34") + krow("s36", "s_add_u32 m0, s34, 1")
    body += row(False, sq, "s35", first_x, second_x, ROWB)
    body += ["s_waitcnt lgkmcnt(0)"]
    body += row(False, sq, "s36", second_x, first_x, 2 * ROWB)
    body += [f"v_add_u32 {AADR}, {2 * ROWB}, {AADR}", "s_waitcnt lgkmcnt(0)"]
    return body


def product(sq):
    e = Emitter()
    e.extend([f"s_mov_b32 {M0_SAVE}, m0"] + load_consts())
    e.extend(load_b_lds(True) if sq else load_b_global())
    e.extend([f"v_mov_b32 {RTHI}, 0", f"v_mov_b32 {RSHI}, 0", f"v_mov_b32 {MASKV}, {MASK}",
              f"v_mov_b32 {AADR}, %[ac]", f"ds_read_b32 {XA[0]}, {AADR}"])
    if not sq:
        e.emit(f"ds_read_b32 {XA[1]}, {AADR} offset:{D1 * ROWB}")
    e.emit("s_waitcnt vmcnt(0) lgkmcnt(0)")
    # row 0 (even: XA), prefetch row 1 into XB
    e.extend(row(True, sq, f"s{KBASE}", XA, XB, ROWB))
    e.extend([f"v_add_u32 {AADR}, {ROWB}, {AADR}", "s_waitcnt lgkmcnt(0)"])
    # rows 1..16: pairs (odd XB, even XA)
    e.extend(["s_mov_b32 s34, 1", "1:"] + pair(sq, XB, XA) +
             ["s_add_u32 s34, s34, 2", f"s_cmp_lg_u32 s34, {MID - 1}", "s_cbranch_scc1 1b"])
    # row 17 (odd: XB), prefetch row 18 into XA
    e.extend(row(False, sq, f"s{KBASE + MID - 1}", XB, XA, ROWB))
    e.extend([f"v_add_u32 {AADR}, {ROWB}, {AADR}"])
    e.extend(mid_reduce())
    e.emit("s_waitcnt lgkmcnt(0)")
    # rows 18..35: pairs (even XA, odd XB)
    e.extend([f"s_mov_b32 s34, {MID}", "2:"] + pair(sq, XA, XB) +
             ["s_add_u32 s34, s34, 2", f"s_cmp_lg_u32 s34, {L}", "s_cbranch_scc1 2b"])
    e.extend(normalise_store())
    e.extend([f"s_mov_b32 m0, {M0_SAVE}", "s_nop 1"])
    return e.out


def row_mads(sq):
    return sum(1 for ln in row(False, sq, "s35", XA, XB, ROWB) if ln.startswith("v_mad_u64_u32"))


def product_mads(sq):
    return L * row_mads(sq) + sum(1 for ln in mid_reduce() if ln.startswith("v_mad_u64_u32"))


def clobbers():
    regs = [f'"v{i}"' for i in range(NREG)]
    regs += [f'"s{i}"' for i in [19, 34, 35, 36] + list(range(KBASE, KBASE + L))]
    out = [", ".join(regs[i:i + 16]) for i in range(0, len(regs), 16)]
    return " \\\n  ".join(x + "," for x in out[:-1]) + " \\\n  " + out[-1]


def c_string(lines):
    return "\n".join(f'  "{ln}\\n"' for ln in lines)


OPERANDS = ", ".join([f'[n{r}] "v"(n[{r}])' for r in range(M)])


def main():
    mm, sq = product(False), product(True)
    hdr = f"""// GENERATED by tools/gen_quad_asm.py -- do not edit by hand.
//
// gfx950 assembly N-adic Montgomery product modulo N^2 over a QUAD of lanes (4 lanes per
// ciphertext, lane l owns limbs 9 l .. 9 l + 8 of both 36-limb digits, radix 2^29,
// R = 2^1044): the LDS column a <- a * b * R^-1 (mod N^2), digits lazily < 2N.
// See tools/gen_quad_asm.py for the layout, the cross-lane steps and the bounds.
// {len(mm)} instructions (general, B from global), {len(sq)} (square); per lane and row
// {row_mads(False)} / {row_mads(True)} v_mad_u64_u32 -> {product_mads(False)} / {product_mads(True)} per product.
#pragma once
#include <stdint.h>

#define FBM_QA_LB {LB}
#define FBM_QA_L {L}
#define FBM_QA_LIMBS {M}
#define FBM_QA_ROWW {ROWW}
#define FBM_QA_ROWB {ROWB}
#define FBM_QA_D1 {D1}
#define FBM_QA_MADS_MUL {product_mads(False)}
#define FBM_QA_MADS_SQR {product_mads(True)}

#define FBM_QA_CLOBBERS \\
  {clobbers()}

// n: the lane's 9 limbs of N (N_(9 l + r)); e0 = (lane % 4 == 0); ac: LDS byte address of the
// ciphertext column (limb 0 of digit 0), al = ac + 9 l * ROWB; QK: the quad constants block
// (K'_i = 2^29 - 1 + K_i, K = (1 - R) mod N, at words 0..35); np = -N^-1 mod 2^29.

// B from global memory, quad layout: limb row j (b0: j = r, b1: j = 9 + r) at
// bb + b_off + j * 1024 (bytes; bb uniform, b_off the lane's offset).
__device__ __forceinline__ void fbm_qa_mm_glb(uint32_t ac, uint32_t al, const uint32_t* bb, uint32_t b_off,
                                              const uint32_t* QK, uint32_t np, const uint32_t (&n)[{M}],
                                              uint32_t e0) {{
  asm volatile(
{c_string(mm)}
      :
      : [ac] "v"(ac), [al] "v"(al), [b] "v"(b_off), [bb] "s"(bb), [QK] "s"(QK), [np] "s"(np), [e0] "v"(e0),
        {OPERANDS}
      : "memory", "vcc", "scc", FBM_QA_CLOBBERS);
}}

// a <- a^2 R^-1 (mod N^2): B = A from the LDS column (the s part as x0 * (2 x1)).
__device__ __forceinline__ void fbm_qa_sq_lds(uint32_t ac, uint32_t al, const uint32_t* QK, uint32_t np,
                                              const uint32_t (&n)[{M}], uint32_t e0) {{
  asm volatile(
{c_string(sq)}
      :
      : [ac] "v"(ac), [al] "v"(al), [QK] "s"(QK), [np] "s"(np), [e0] "v"(e0),
        {OPERANDS}
      : "memory", "vcc", "scc", FBM_QA_CLOBBERS);
}}
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}: general {len(mm)} / square {len(sq)} instructions; mads/row {row_mads(False)} / "
          f"{row_mads(True)}")


if __name__ == "__main__":
    main()
