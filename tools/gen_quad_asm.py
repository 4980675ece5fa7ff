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

TRIPLE variant (G = 3 lanes per ciphertext, 12 limbs per lane, fbm_tri_asm.hpp): 21
ciphertexts per wave (lanes 0..62) + one dummy lane (63, all-zero data).  Same arithmetic and
register roles; the cross-lane steps cannot use quad_perm (groups of 3 straddle the 4-lane DPP
quads), so
  * the quotient digits are masked in place (v_and_b32) and broadcast from the group's lane 0
    by ds_bpermute_b32 (an LDS-pipe op: no VALU cycle; its latency hides behind the row's
    multiplies -- s_waitcnt lgkmcnt before the first use), lane 0 itself using its own copy;
  * the retire rotation (lane -> lane below) is v_and_b32_dpp wave_shl:1 bound_ctrl:0 (the
    group's top lane receives the next group's lane 0, whose masked value is 0; lane 62
    receives the dummy's 0), the carry hand-ups are v_mov_b32_dpp wave_shr:1 bound_ctrl:0.
Why: a launch of n ciphertexts needs ceil(n / 16) quad waves but ceil(n / 21) triple waves;
at a config-4 stripe (41 667) that is 2.54 vs 1.94 waves per SIMD, i.e. 3 vs 2 on the
busiest SIMD, and one triple wave costs ~1.16 quad waves.

Usage:  python tools/gen_quad_asm.py   (rewrites both headers; the build does not run this)
"""

import os

LB = 29         # bits per limb
L = 36          # limbs per digit
MID = 18        # rows before the mid-product reduction
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MASK = hex((1 << LB) - 1)


class Geo:
    """Register plan and cross-lane primitives of one engine: G lanes per ciphertext,
    M = 36 / G limbs per lane."""

    def __init__(self, G, rows_w):
        self.G, self.M = G, L // G
        self.ROWW, self.ROWB, self.D1 = rows_w, rows_w * 4, L
        M = self.M
        self.TT0 = 2 * (M - 1)          # t window: slots 0..M-2 at v[0:2M-3], TT, RT
        self.RT0 = self.TT0 + 2
        self.AS0 = self.RT0 + 2         # s window
        self.TS0 = self.AS0 + 2 * (M - 1)
        self.RS0 = self.TS0 + 2
        self.B00 = self.RS0 + 2         # b0[0..M-1], b1[0..M-1]
        self.B10 = self.B00 + M
        x = self.B10 + M
        self.XA, self.XB = (f"v{x}", f"v{x + 1}"), (f"v{x + 2}", f"v{x + 3}")
        names = ["Q", "Q2", "CQ", "AADR", "TMP", "TMP2", "MASKV"]
        for i, nm in enumerate(names):
            setattr(self, nm, f"v{x + 4 + i}")
        c = x + 4 + len(names) + 1      # (quad: one spare register before the carry pairs)
        self.CY, self.CYLO, self.CYHI = f"v[{c}:{c + 1}]", f"v{c}", f"v{c + 1}"
        self.CS, self.CSLO, self.CSHI = f"v[{c + 2}:{c + 3}]", f"v{c + 2}", f"v{c + 3}"
        self.T3, self.T4 = f"v{c + 4}", f"v{c + 5}"
        nreg = c + 6
        if G == 3:                      # broadcast copies of the quotient digits
            self.QB, self.Q2B = f"v{nreg}", f"v{nreg + 1}"
            nreg += 2
        else:
            self.QB, self.Q2B = self.Q, self.Q2
        self.NREG = nreg
        self.TT, self.TTLO = f"v[{self.TT0}:{self.TT0 + 1}]", f"v{self.TT0}"
        self.RT, self.RTLO, self.RTHI = f"v[{self.RT0}:{self.RT0 + 1}]", f"v{self.RT0}", f"v{self.RT0 + 1}"
        self.TS, self.TSLO = f"v[{self.TS0}:{self.TS0 + 1}]", f"v{self.TS0}"
        self.RS, self.RSLO, self.RSHI = f"v[{self.RS0}:{self.RS0 + 1}]", f"v{self.RS0}", f"v{self.RS0 + 1}"

    def At(self, k):
        return f"v[{2 * k}:{2 * k + 1}]"

    def AtLo(self, k):
        return f"v{2 * k}"

    def AtHi(self, k):
        return f"v{2 * k + 1}"

    def As(self, k):
        return f"v[{self.AS0 + 2 * k}:{self.AS0 + 2 * k + 1}]"

    def AsLo(self, k):
        return f"v{self.AS0 + 2 * k}"

    def AsHi(self, k):
        return f"v{self.AS0 + 2 * k + 1}"

    def B0(self, r):
        return f"v{self.B00 + r}"

    def B1(self, r):
        return f"v{self.B10 + r}"

    # ---- cross-lane steps ----
    def down(self, op, dst, src, extra=""):
        """dst <- src of the lane above (the lane below receives): retire rotation"""
        if self.G == 4:
            return f"{op} {dst}, {src}{extra} {dpp((1, 2, 3, 0))}"
        return f"{op} {dst}, {src}{extra} wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"

    def up(self, dst, src):
        """dst <- src of the lane below (carry hand-up; the group's lane 0 receives 0)"""
        if self.G == 4:
            return f"v_mov_b32_dpp {dst}, {src} {dpp((3, 0, 1, 2))}"
        return f"v_mov_b32_dpp {dst}, {src} wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"


# Round 4 experiment: the triple's quotient broadcasts on the VALU instead of the LDS pipe.  The
# quotient digit is masked with a lane-dependent mask (%[mq] = 2^29 - 1 in a group's lane 0, 0 in the
# others), so a group holds one nonzero copy, and two DPP adds over wave_shr:1 sum it into every lane
# of the group: QT = Q(i-1) + Q(i), QB = QT(i-1) + Q(i) = Q(i-2) + Q(i-1) + Q(i) -- the value of the
# group's lane 0 in lanes 0, 1, 2 (the neighbours' copies are 0; lane 0 of the wave reads 0 past the
# end).  Two VALU instructions per broadcast in place of one ds_bpermute and its LDS latency.
# Measured equal to the permutes alone and 1 % slower with CYC_B0D (profiles/archive/r4_tri_dpp_ab.jsonl,
# r4_tri_b0d_ab.jsonl): the 144 extra VALU instructions per square cost what the permutes' LDS latency did.
TRI_DPP_BCAST = os.environ.get("FBM_GEN_TRI_DPP", "0") == "1"  # (an A/B switch, off)

QUAD = Geo(4, 72)   # 64 ciphertexts per workgroup + 8 words of padding
TRI = Geo(3, 89)    # 84 ciphertexts + the dummy column + 4 words of padding


def dpp_bcast(dst, tmp, src):
    """The triple's group broadcast of a lane-masked value (TRI_DPP_BCAST): two DPP adds."""
    sh = "wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
    return [f"v_add_u32_dpp {tmp}, {src}, {src} {sh}", f"v_add_u32_dpp {dst}, {tmp}, {src} {sh}"]


def tri_chain(q, q2, qb, q2b, t3, t4, tlo, slo, spair, cq, kreg):
    """The triple's quotient chain: q from the t column's low word, the s column's K'_i - q, q' from the
    s column; the broadcasts by ds_bpermute or two DPP adds (TRI_DPP_BCAST).  Returns the instructions
    and, for each after the first, the independent multiplies to place before it."""
    fix, fgap = [f"v_sub_u32 {cq}, {kreg}, {q}", f"v_mad_u64_u32 {spair}, vcc, {cq}, %[e0], {spair}"], [2, 2]
    if TRI_DPP_BCAST:
        chain = ([f"v_mul_lo_u32 {q}, {tlo}, %[np]", f"v_and_b32 {q}, %[mq], {q}"] + fix + dpp_bcast(qb, t3, q) +
                 [f"v_mul_lo_u32 {q2}, {slo}, %[np]", f"v_and_b32 {q2}, %[mq], {q2}"] + dpp_bcast(q2b, t4, q2))
        gaps = [2] + [1] * len(fix) + [1, 2, 1, 2, 2, 2]
    else:
        chain = ([f"v_mul_lo_u32 {q}, {tlo}, %[np]", f"v_and_b32 {q}, {MASK}, {q}",
                  f"ds_bpermute_b32 {qb}, %[bp], {q}"] + fix +
                 [f"v_mul_lo_u32 {q2}, {slo}, %[np]", f"v_and_b32 {q2}, {MASK}, {q2}",
                  f"ds_bpermute_b32 {q2b}, %[bp], {q2}"])
        gaps = [2, 0] + fgap + [3, 2, 0]
    return chain, gaps


def N(r):
    return f"%[n{r}]"


def dpp(perm):
    return f"quad_perm:[{','.join(str(p) for p in perm)}] row_mask:0xf bank_mask:0xf"


def is_dpp(ln):
    return "quad_perm" in ln or "wave_sh" in ln


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
        if is_dpp(ln):
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


def load_b_global(g):
    """b0[r] = limb row r, b1[r] = limb row M + r of the lane's table column: word
    (row * 256 + lane) of the block, rows 1 KB apart (%[b] = the lane's byte offset from the
    uniform %[bb])."""
    out = ["s_waitcnt vmcnt(0)", f"v_mov_b32 {g.TMP}, %[b]"]
    for j in range(2 * g.M):
        if j and j % 4 == 0:
            out.append(f"v_add_u32 {g.TMP}, 0x1000, {g.TMP}")
        reg = g.B0(j) if j < g.M else g.B1(j - g.M)
        out.append(f"global_load_dword {reg}, {g.TMP}, %[bb] offset:{(j % 4) * 1024}")
    return out


def load_b_lds(g, double_b1):
    out = []
    for r in range(g.M):
        out.append(f"ds_read_b32 {g.B0(r)}, %[al] offset:{r * g.ROWB}")
        out.append(f"ds_read_b32 {g.B1(r)}, %[al] offset:{(g.D1 + r) * g.ROWB}")
    out.append("s_waitcnt lgkmcnt(0)")
    if double_b1:  # square: the s part is x0 * (2 x1)
        out += [f"v_lshlrev_b32 {g.B1(r)}, 1, {g.B1(r)}" for r in range(g.M)]
    return out


def row(g, first, sq, kreg, xs, xn, pre_off, first_s=None):
    """One row with an explicit schedule (every dependent instruction 3+ instructions after
    its producer).  xs = this row's (x0, x1); xn = where the prefetch of the next row's
    operands goes, read at byte offset pre_off from AADR; kreg = K'_i.  first_s (default: first):
    whether the s window starts from 0 (False: from its registers -- the short product's D)."""
    M = g.M
    x0, x1 = xs
    first_s = first if first_s is None else first_s
    out = [f"ds_read_b32 {xn[0]}, {g.AADR} offset:{pre_off}"]
    if not sq:
        out.append(f"ds_read_b32 {xn[1]}, {g.AADR} offset:{pre_off + g.D1 * g.ROWB}")

    def addend(acc, r):
        if first if acc == g.At else first_s:
            return "0"
        if r == M - 1:
            return g.RT if acc == g.At else g.RS
        return acc(r)

    def tm(r):  # t pass 1: x0 * b0[r]
        dst = g.TT if r == 0 else g.At(r - 1)
        return f"v_mad_u64_u32 {dst}, vcc, {x0}, {g.B0(r)}, {addend(g.At, r)}"

    def sm(r):  # s pass 1: x0 * b1[r]
        dst = g.TS if r == 0 else g.As(r - 1)
        return f"v_mad_u64_u32 {dst}, vcc, {x0}, {g.B1(r)}, {addend(g.As, r)}"

    # ---- pass 1: x0_i * b0 (t) and x0_i * b1 (s), the quotient chains threaded through ----
    if g.G == 4:
        Q, Q2, CQ, MASKV, TSLO, TTLO, TS = g.Q, g.Q2, g.CQ, g.MASKV, g.TSLO, g.TTLO, g.TS
        p1 = [tm(0), sm(0), tm(1)]
        if not sq:
            p1.append(f"v_mad_u64_u32 {TS}, vcc, {x1}, {g.B0(0)}, {TS}")
        p1 += [tm(2), f"v_mul_lo_u32 {Q}, {TTLO}, %[np]", sm(1), tm(3), sm(2),
               f"v_and_b32_dpp {Q}, {Q}, {MASKV} {dpp((0, 0, 0, 0))}", sm(3), tm(4),
               f"v_sub_u32 {CQ}, {kreg}, {Q}", sm(4), tm(5),      # K'_i - q (>= 0: K'_i >= 2^29 - 1)
               f"v_mad_u64_u32 {TS}, vcc, {CQ}, %[e0], {TS}", sm(5), tm(6),
               f"v_mul_lo_u32 {Q2}, {TSLO}, %[np]", sm(6), tm(7), sm(7),
               f"v_and_b32_dpp {Q2}, {Q2}, {MASKV} {dpp((0, 0, 0, 0))}", tm(8), sm(8)]
    else:
        # the same chain with the broadcasts on the LDS pipe: lane 0 subtracts its own masked q;
        # the others take the group's q from lane 0 by ds_bpermute (QB / Q2B, waited for below)
        mads = [tm(0), sm(0), tm(1)] + ([] if sq else [f"v_mad_u64_u32 {g.TS}, vcc, {x1}, {g.B0(0)}, {g.TS}"])
        rest = []
        for r in range(2, M):
            rest += [tm(r), sm(r - 1)]
        rest.append(sm(M - 1))
        chain, gaps = tri_chain(g.Q, g.Q2, g.QB, g.Q2B, g.T3, g.T4, g.TTLO, g.TSLO, g.TS, g.CQ, kreg)
        gaps = [1] + gaps
        p1 = list(mads)
        ri = 0
        for k, ins in enumerate(chain):
            take = gaps[k] if k else max(0, 3 - (len(mads) - 1))
            p1 += rest[ri:ri + take]
            ri += take
            p1.append(ins)
        p1 += rest[ri:]
        if not TRI_DPP_BCAST:
            p1.append("s_waitcnt lgkmcnt(1)")  # QB (the Q2B permute may still be in flight)
    # ---- pass 2: q * N (t), interleaved with x1_i * b0 (s, general product) ----
    tq = [f"v_mad_u64_u32 {g.TT}, vcc, {g.QB}, {N(0)}, {g.TT}"] + \
        [f"v_mad_u64_u32 {g.At(r - 1)}, vcc, {g.QB}, {N(r)}, {g.At(r - 1)}" for r in range(1, M)]
    sx = [] if sq else [f"v_mad_u64_u32 {g.As(r - 1)}, vcc, {x1}, {g.B0(r)}, {g.As(r - 1)}" for r in range(1, M)]
    p2 = []
    for k in range(max(len(tq), len(sx))):
        if k < len(tq):
            p2.append(tq[k])
        if k < len(sx):
            p2.append(sx[k])
    # ---- pass 3: q' * N (s), both retires threaded in:
    #      T = lo + c 2^29 -> lo (masked) to the lane below's top slot, c into the new slot 0 ----
    sq3 = [f"v_mad_u64_u32 {g.TS}, vcc, {g.Q2B}, {N(0)}, {g.TS}"] + \
        [f"v_mad_u64_u32 {g.As(r - 1)}, vcc, {g.Q2B}, {N(r)}, {g.As(r - 1)}" for r in range(1, M)]
    ret_t = [g.down("v_and_b32_dpp", g.RTLO, g.TTLO, f", {g.MASKV}"),
             f"v_lshrrev_b64 {g.TT}, {LB}, {g.TT}",
             f"v_lshl_add_u64 {g.At(0)}, {g.TT}, 0, {g.At(0)}"]
    ret_s = [g.down("v_and_b32_dpp", g.RSLO, g.TSLO, f", {g.MASKV}"),
             f"v_lshrrev_b64 {g.TS}, {LB}, {g.TS}",
             f"v_lshl_add_u64 {g.As(0)}, {g.TS}, 0, {g.As(0)}"]
    p3 = [] if (g.G == 4 or TRI_DPP_BCAST) else ["s_waitcnt lgkmcnt(0)"]
    p3 += [sq3[0], ret_t[0], sq3[1], ret_t[1], sq3[2], ret_t[2], sq3[3], ret_s[0], sq3[4], ret_s[1], sq3[5],
           ret_s[2]] + sq3[6:]
    return out + p1 + p2 + p3


# Round 4: no mid-product reduction in the group engines.  A column lives in a lane's window for at
# most M rows: the row that retires a lane's slot 0 hands only its low 29 bits to the lane below (the
# carry stays, in slot 1), so every column restarts from < 2^29 whenever it changes lanes -- at most M
# rows of products (12 in the triple: 12 x 3 x 2^58 < 2^64) -- tests/asm_bounds.py proves every 64-bit
# multiply-add below 2^64 for every operand within the products' bounds without it (the round-3
# engines carried the one-lane engine's pass after row 17: ~50 VALU instructions per product).
GROUP_MID_REDUCE = False


def mid_reduce(g):
    """(Unused unless GROUP_MID_REDUCE.)  After row 17: every slot keeps its low dword and hands the high one to the slot above
    (x 8 = 2^32 / 2^29); the top slot's (R) high dword goes to the lane above's slot 0
    (the top lane's is 0: the window's value is below 2^1026).  Values drop below 2^36."""
    M = g.M
    if not GROUP_MID_REDUCE:
        return []
    chains = []
    for acc, hi, rr, rhi, t in ((g.At, g.AtHi, g.RT, g.RTHI, g.T3), (g.As, g.AsHi, g.RS, g.RSHI, g.T4)):
        ch = []
        for k in range(M - 2):
            ch += [f"v_mad_u64_u32 {acc(k + 1)}, vcc, {hi(k)}, 8, {acc(k + 1)}", f"v_mov_b32 {hi(k)}, 0"]
        ch += [f"v_mad_u64_u32 {rr}, vcc, {hi(M - 2)}, 8, {rr}", f"v_mov_b32 {hi(M - 2)}, 0",
               g.up(t, rhi),
               f"v_mov_b32 {rhi}, 0",
               f"v_mad_u64_u32 {acc(0)}, vcc, {t}, 8, {acc(0)}"]
        chains.append(ch)
    out = []
    for a, b in zip(*chains):
        out += [a, b]
    return out


def normalise_store(g):
    """Window (slots 0..M-2 + R) -> M lazy 29-bit limbs per digit part, into the b registers
    (t -> b0, s -> b1), and the lane's slice of the LDS column.  The t and s carry chains are
    independent: interleaved instruction by instruction (a vcc add/addc pair kept together)."""
    M = g.M
    chains = []
    for acc, lo, rr, rlo, breg, cy, cylo, cyhi, t1, t2 in (
            (g.At, g.AtLo, g.RT, g.RTLO, g.B0, g.CY, g.CYLO, g.CYHI, g.TMP, g.TMP2),
            (g.As, g.AsLo, g.RS, g.RSLO, g.B1, g.CS, g.CSLO, g.CSHI, g.T3, g.T4)):
        ch = [f"v_and_b32 {breg(0)}, {MASK}, {lo(0)}", f"v_lshrrev_b64 {cy}, {LB}, {acc(0)}"]
        for r in range(1, M - 1):
            ch += [f"v_lshl_add_u64 {acc(r)}, {cy}, 0, {acc(r)}",
                   f"v_and_b32 {breg(r)}, {MASK}, {lo(r)}",
                   f"v_lshrrev_b64 {cy}, {LB}, {acc(r)}"]
        ch += [f"v_lshl_add_u64 {rr}, {cy}, 0, {rr}",
               f"v_and_b32 {breg(M - 1)}, {MASK}, {rlo}",
               f"v_lshrrev_b64 {cy}, {LB}, {rr}",
               # carry-out -> the lane above (the group's lane 0 receives the top lane's, which is 0)
               g.up(t1, cylo),
               g.up(t2, cyhi),
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
    for d, breg in ((0, g.B0), (1, g.B1)):
        out += [f"ds_write_b32 %[al], {breg(r)} offset:{(d * g.D1 + r) * g.ROWB}" for r in range(M)]
    out.append("s_waitcnt lgkmcnt(0)")
    return out


KBASE = 64      # K'_i in s(64 + i)
M0_SAVE = "s19"


def krow(dst, m0_expr):
    """dst <- K'_row (s_movrels after an SALU write of m0 needs a wait state)."""
    return [m0_expr, "s_nop 1", f"s_movrels_b32 {dst}, s{KBASE}"]


def pair(g, sq, first_x, second_x):
    """Rows (i, i+1) with i = s34; operands of row i in first_x, of row i+1 in second_x."""
    body = krow("s35", "s_mov_b32 m0, s34") + krow("s36", "s_add_u32 m0, s34, 1")
    body += row(g, False, sq, "s35", first_x, second_x, g.ROWB)
    body += ["s_waitcnt lgkmcnt(0)"]
    body += row(g, False, sq, "s36", second_x, first_x, 2 * g.ROWB)
    body += [f"v_add_u32 {g.AADR}, {2 * g.ROWB}, {g.AADR}", "s_waitcnt lgkmcnt(0)"]
    return body


CARRY_PAIRS = ("vcc", "s[20:21]")  # the mads' (never read) carry-outs, alternated: see rotate_carries


def rotate_carries(lines, pairs=CARRY_PAIRS):
    """Alternate the carry-out destination of successive v_mad_u64_u32 over `pairs`.  Every mad
    writing vcc chains a wave's mads through one SGPR pair (write-after-write): a wave then issues
    one every ~8.8 clocks; two pairs in turn cut that to ~5.8 (tools/microbench/gen_oprate.py) and a
    triple-engine square by 15 % at two waves per SIMD (tools/microbench/tri_variants.py)."""
    out, i = [], 0
    for ln in lines:
        if ln.startswith("v_mad_u64_u32") and ", vcc," in ln:
            ln = ln.replace(", vcc,", f", {pairs[i % len(pairs)]},", 1)
            i += 1
        out.append(ln)
    return out


def product(sq, g=QUAD, carries=CARRY_PAIRS, cyc=None):
    if sq and (CYC_SQUARE if cyc is None else cyc):
        return square_cyc(g, carries)
    e = Emitter()
    XA, XB = g.XA, g.XB
    e.extend([f"s_mov_b32 {M0_SAVE}, m0"] + load_consts())
    e.extend(load_b_lds(g, True) if sq else load_b_global(g))
    e.extend([f"v_mov_b32 {g.RTHI}, 0", f"v_mov_b32 {g.RSHI}, 0", f"v_mov_b32 {g.MASKV}, {MASK}",
              f"v_mov_b32 {g.AADR}, %[ac]", f"ds_read_b32 {XA[0]}, {g.AADR}"])
    if not sq:
        e.emit(f"ds_read_b32 {XA[1]}, {g.AADR} offset:{g.D1 * g.ROWB}")
    e.emit("s_waitcnt vmcnt(0) lgkmcnt(0)")
    # row 0 (even: XA), prefetch row 1 into XB
    e.extend(row(g, True, sq, f"s{KBASE}", XA, XB, g.ROWB))
    e.extend([f"v_add_u32 {g.AADR}, {g.ROWB}, {g.AADR}", "s_waitcnt lgkmcnt(0)"])
    # rows 1..16: pairs (odd XB, even XA)
    e.extend(["s_mov_b32 s34, 1", "1:"] + pair(g, sq, XB, XA) +
             ["s_add_u32 s34, s34, 2", f"s_cmp_lg_u32 s34, {MID - 1}", "s_cbranch_scc1 1b"])
    # row 17 (odd: XB), prefetch row 18 into XA
    e.extend(row(g, False, sq, f"s{KBASE + MID - 1}", XB, XA, g.ROWB))
    e.extend([f"v_add_u32 {g.AADR}, {g.ROWB}, {g.AADR}"])
    e.extend(mid_reduce(g))
    e.emit("s_waitcnt lgkmcnt(0)")
    # rows 18..35: pairs (even XA, odd XB)
    e.extend([f"s_mov_b32 s34, {MID}", "2:"] + pair(g, sq, XA, XB) +
             ["s_add_u32 s34, s34, 2", f"s_cmp_lg_u32 s34, {L}", "s_cbranch_scc1 2b"])
    e.extend(normalise_store(g))
    e.extend([f"s_mov_b32 m0, {M0_SAVE}", "s_nop 1"])
    return rotate_carries(e.out, carries)


# ------------------------------------------------------------------------------------------
# The square as a cyclic-band triangular product (round 3).  x0^2 needs each cross product
# x_a x_b (a < b) once, doubled, and each diagonal x_a^2 once.  Row i's t part multiplies x_i by
# the lane's b-limbs j = M l + r; whether a product is needed depends only on
# rho = (j - i) mod M = (r - i) mod M -- the same in every lane of the group, so one instruction
# stream serves all lanes: rho in 1..ceil(M/2)-1 with 2 x_i (the pair's mirror, rho' = M - rho,
# is skipped in row j), rho = 0 and rho = M/2 with x_i undoubled (their pairs come up in both
# rows: twice, undoubled; rho = 0 within a row's own column is the diagonal, once).  7 of 12 t
# products per lane and row in the triple, 5 of 9 in the quad (49 -> 44 / 37 -> 33 multiplies).
# Which registers a row multiplies changes with i mod M, so the 36 rows are unrolled; the window
# shift is static register renaming over M + 1 pairs per digit part (slot r of row i in pair
# (i + r) mod (M + 1)), every product accumulating in place; the received top slot arrives in RT /
# RS (hi 0) and is taken in by the top slot's first product of the next row (as addend).  The
# K'_i are read from s(64 + i) directly (no m0).  Same residues as the looped square.
# ------------------------------------------------------------------------------------------
CYC_SQUARE = True
# Round 4: the cyclic-band square's doubled cross products as x_i * (2 b0[r]) from M doubled limb
# registers made once per square, in place of 2 x_i made once per row (36 -> M shifts per square): the
# triple at one rank's 1/8 / 1/4 stripe -0.7 / -1.2 % (profiles/archive/r4_tri_b0d_ab.jsonl).  FBM_GEN_CYC_B0D=0
# generates the per-row doubling (the A/B base).
CYC_B0D = os.environ.get("FBM_GEN_CYC_B0D", "1") == "1"


class CycPlan:
    """Register plan of square_cyc for geometry g (pairs named by their low VGPR)."""

    def __init__(self, g):
        M = g.M
        self.W = W = M + 1
        v = 0
        self.PT = [v + 2 * k for k in range(W)]
        v += 2 * W
        self.RT = v
        v += 2
        self.PS = [v + 2 * k for k in range(W)]
        v += 2 * W
        self.RS = v
        v += 2
        self.B0 = [v + r for r in range(M)]
        v += M
        self.B1 = [v + r for r in range(M)]
        v += M
        if CYC_B0D:
            self.B0D = [v + r for r in range(M)]
            v += M
        self.X = (v, v + 1)  # x0 of even / odd rows
        self.XD = v + 2      # 2 x0 of the current row
        v += 3
        for nm in ("Q", "Q2", "CQ", "MASKV", "QB", "Q2B", "T3", "T4", "TMP", "TMP2"):
            setattr(self, nm, v)
            v += 1
        v += v % 2  # 64-bit pairs start on an even VGPR
        self.CY, self.CS = v, v + 2
        v += 4
        self.NREG = v


def _pr(lo):
    return f"v[{lo}:{lo + 1}]"


def cyc_active(g, i):
    """[(r, doubled)] of row i's t products (see above)."""
    M = g.M
    out = []
    for r in range(M):
        rho = (r - i) % M
        if rho == 0 or (M % 2 == 0 and rho == M // 2):
            out.append((r, False))
        elif 1 <= rho <= (M - 1) // 2:
            out.append((r, True))
    return out


def cyc_row(g, P, i):
    M, W = g.M, P.W
    first, last = i == 0, i == L - 1
    xs, xn = P.X[i % 2], P.X[(i + 1) % 2]
    st = lambda r: P.PT[(i + r) % W]  # noqa: E731
    ss = lambda r: P.PS[(i + r) % W]  # noqa: E731
    touched = {"t": set(), "s": set()}

    def addend(part, r):
        reg = st(r) if part == "t" else ss(r)
        if r in touched[part]:
            return _pr(reg)
        touched[part].add(r)
        if first:
            return "0"
        if r == M - 1:
            return _pr(P.RT if part == "t" else P.RS)
        return _pr(reg)

    out = [] if last else [f"ds_read_b32 v{xn}, %[ac] offset:{(i + 1) * g.ROWB}"]
    acts = cyc_active(g, i)
    if CYC_B0D:
        tm = {r: f"v_mad_u64_u32 {_pr(st(r))}, vcc, v{xs}, v{P.B0D[r] if dbl else P.B0[r]}, {addend('t', r)}"
              for r, dbl in acts}
    else:
        tm = {r: f"v_mad_u64_u32 {_pr(st(r))}, vcc, v{P.XD if dbl else xs}, v{P.B0[r]}, {addend('t', r)}"
              for r, dbl in acts}
    sm = [f"v_mad_u64_u32 {_pr(ss(r))}, vcc, v{xs}, v{P.B1[r]}, {addend('s', r)}" for r in range(M)]
    # pass 1: slot 0's t and s products first, the rest interleaved; the quotient chain threaded in
    head = ([tm[0]] if 0 in tm else []) + [sm[0]]
    t_rest = [tm[r] for r, _ in acts if r != 0]
    s_rest = sm[1:]
    rest = []
    for k in range(max(len(t_rest), len(s_rest))):
        if k < len(t_rest):
            rest.append(t_rest[k])
        if k < len(s_rest):
            rest.append(s_rest[k])
    K = f"s{KBASE + i}"
    if g.G == 4:
        chain = [f"v_mul_lo_u32 v{P.Q}, v{st(0)}, %[np]",
                 f"v_and_b32_dpp v{P.Q}, v{P.Q}, v{P.MASKV} {dpp((0, 0, 0, 0))}",
                 f"v_sub_u32 v{P.CQ}, {K}, v{P.Q}",
                 f"v_mad_u64_u32 {_pr(ss(0))}, vcc, v{P.CQ}, %[e0], {_pr(ss(0))}",
                 f"v_mul_lo_u32 v{P.Q2}, v{ss(0)}, %[np]",
                 f"v_and_b32_dpp v{P.Q2}, v{P.Q2}, v{P.MASKV} {dpp((0, 0, 0, 0))}"]
        gaps = [1 if 0 in tm else 0, 2, 2, 2, 3, 2]
        qb, q2b = P.Q, P.Q2
    else:
        chain, gaps = tri_chain(f"v{P.Q}", f"v{P.Q2}", f"v{P.QB}", f"v{P.Q2B}", f"v{P.T3}", f"v{P.T4}",
                                f"v{st(0)}", f"v{ss(0)}", _pr(ss(0)), f"v{P.CQ}", K)
        gaps = [1 if 0 in tm else 0] + gaps
        qb, q2b = P.QB, P.Q2B
    p1 = list(head)
    ri = 0
    for k, ins in enumerate(chain):
        take = gaps[k]
        p1 += rest[ri:ri + take]
        ri += take
        p1.append(ins)
    p1 += rest[ri:]
    if g.G == 3 and not TRI_DPP_BCAST:
        p1.append("s_waitcnt lgkmcnt(1)")  # the row prefetch and QB (Q2B may still be in flight)
    # pass 2: q N into the t window
    p2 = [f"v_mad_u64_u32 {_pr(st(r))}, vcc, v{qb}, {N(r)}, {addend('t', r)}" for r in range(M)]
    # pass 3: q' N into the s window, both retires threaded in:
    #   T = lo + c 2^29 -> lo (masked) to the lane below's top slot (RT / RS), c into slot 1
    sq3 = [f"v_mad_u64_u32 {_pr(ss(r))}, vcc, v{q2b}, {N(r)}, {addend('s', r)}" for r in range(M)]
    ret_t = [g.down("v_and_b32_dpp", f"v{P.RT}", f"v{st(0)}", f", v{P.MASKV}"),
             f"v_lshrrev_b64 {_pr(st(0))}, {LB}, {_pr(st(0))}",
             f"v_lshl_add_u64 {_pr(st(1))}, {_pr(st(0))}, 0, {_pr(st(1))}"]
    ret_s = [g.down("v_and_b32_dpp", f"v{P.RS}", f"v{ss(0)}", f", v{P.MASKV}"),
             f"v_lshrrev_b64 {_pr(ss(0))}, {LB}, {_pr(ss(0))}",
             f"v_lshl_add_u64 {_pr(ss(1))}, {_pr(ss(0))}, 0, {_pr(ss(1))}"]
    early = (g.G == 3 and not TRI_DPP_BCAST) or not CYC_B0D  # Q2B (bpermute) or the XD shift need xn / q' now
    p3 = ["s_waitcnt lgkmcnt(0)"] if early else []
    if not last and not CYC_B0D:  # the next row's doubled operand (its x0 has arrived with the wait above)
        p3.append(f"v_lshlrev_b32 v{P.XD}, 1, v{xn}")
    p3 += [sq3[0], ret_t[0], sq3[1], ret_t[1], sq3[2], ret_t[2], sq3[3], ret_s[0], sq3[4], ret_s[1], sq3[5],
           ret_s[2]] + sq3[6:]
    if not early:  # the next row's operand, prefetched above
        p3.append("s_waitcnt lgkmcnt(0)")
    return out + p1 + p2 + p3


CYC_MID_KEEP = {}  # geometry name -> (t slots, s slots) reduced ("R": the top slot's hand-up); absent: all


def cyc_mid_reduce(g, P, i):
    """mid_reduce with the window of row i (slots 0..M-2 in their pairs, the top slot in RT / RS).
    CYC_MID_KEEP[g]: per part the slots that need it (k: slot k's high dword into slot k + 1; "R": the
    top slot's into the lane above's slot 0) -- the rest provably stay below 2^64 without
    (tests/asm_bounds.py)."""
    M, W = g.M, P.W
    if not GROUP_MID_REDUCE:
        return []
    keep = CYC_MID_KEEP.get("triple" if g.G == 3 else "quad")
    chains = []
    for part, (pt, rr, t) in enumerate(((P.PT, P.RT, P.T3), (P.PS, P.RS, P.T4))):
        acc = lambda k, pt=pt: pt[(i + k) % W]  # noqa: E731
        kp = None if keep is None else keep[part]
        ch = []
        for k in range(M - 2):
            if kp is None or k in kp:
                ch += [f"v_mad_u64_u32 {_pr(acc(k + 1))}, vcc, v{acc(k) + 1}, 8, {_pr(acc(k + 1))}",
                       f"v_mov_b32 v{acc(k) + 1}, 0"]
        if kp is None or M - 2 in kp:
            ch += [f"v_mad_u64_u32 {_pr(rr)}, vcc, v{acc(M - 2) + 1}, 8, {_pr(rr)}", f"v_mov_b32 v{acc(M - 2) + 1}, 0"]
        if kp is None or "R" in kp:
            ch += [g.up(f"v{t}", f"v{rr + 1}"),
                   f"v_mov_b32 v{rr + 1}, 0",
                   f"v_mad_u64_u32 {_pr(acc(0))}, vcc, v{t}, 8, {_pr(acc(0))}"]
        chains.append(ch)
    out = []
    for k in range(max(len(c) for c in chains)):
        for ch in chains:
            if k < len(ch):
                out.append(ch[k])
    return out


def cyc_normalise_store(g, P):
    """normalise_store with the window after row 35 (slots 0..M-2 in their pairs, the top in RT / RS)."""
    M, W = g.M, P.W
    i = L
    chains = []
    for pt, rr, breg, cy, t1, t2 in ((P.PT, P.RT, P.B0, P.CY, P.TMP, P.TMP2), (P.PS, P.RS, P.B1, P.CS, P.T3, P.T4)):
        acc = lambda k, pt=pt: pt[(i + k) % W]  # noqa: E731
        ch = [f"v_and_b32 v{breg[0]}, {MASK}, v{acc(0)}", f"v_lshrrev_b64 {_pr(cy)}, {LB}, {_pr(acc(0))}"]
        for r in range(1, M - 1):
            ch += [f"v_lshl_add_u64 {_pr(acc(r))}, {_pr(cy)}, 0, {_pr(acc(r))}",
                   f"v_and_b32 v{breg[r]}, {MASK}, v{acc(r)}",
                   f"v_lshrrev_b64 {_pr(cy)}, {LB}, {_pr(acc(r))}"]
        ch += [f"v_lshl_add_u64 {_pr(rr)}, {_pr(cy)}, 0, {_pr(rr)}",
               f"v_and_b32 v{breg[M - 1]}, {MASK}, v{rr}",
               f"v_lshrrev_b64 {_pr(cy)}, {LB}, {_pr(rr)}",
               g.up(f"v{t1}", f"v{cy}"),
               g.up(f"v{t2}", f"v{cy + 1}"),
               f"v_add_co_u32 v{t1}, vcc, v{t1}, v{breg[0]}|v_addc_co_u32 v{t2}, vcc, 0, v{t2}, vcc",
               f"v_and_b32 v{breg[0]}, {MASK}, v{t1}",
               f"v_alignbit_b32 v{t1}, v{t2}, v{t1}, {LB}",
               f"v_add_u32 v{breg[1]}, v{breg[1]}, v{t1}"]
        chains.append(ch)
    out = []
    for k in range(max(len(c) for c in chains)):
        for ch in chains:
            if k < len(ch):
                out += ch[k].split("|")
    for d, breg in ((0, P.B0), (1, P.B1)):
        out += [f"ds_write_b32 %[al], v{breg[r]} offset:{(d * g.D1 + r) * g.ROWB}" for r in range(M)]
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def square_cyc(g, carries=CARRY_PAIRS):
    P = CycPlan(g)
    M = g.M
    e = Emitter()
    e.extend(load_consts())
    for r in range(M):
        e.emit(f"ds_read_b32 v{P.B0[r]}, %[al] offset:{r * g.ROWB}")
        e.emit(f"ds_read_b32 v{P.B1[r]}, %[al] offset:{(g.D1 + r) * g.ROWB}")
    e.extend([f"v_mov_b32 v{P.RT + 1}, 0", f"v_mov_b32 v{P.RS + 1}, 0", f"v_mov_b32 v{P.MASKV}, {MASK}",
              f"ds_read_b32 v{P.X[0]}, %[ac]", "s_waitcnt lgkmcnt(0)"])
    e.extend([f"v_lshlrev_b32 v{P.B1[r]}, 1, v{P.B1[r]}" for r in range(M)])  # the s part is x0 * (2 x1)
    if CYC_B0D:
        e.extend([f"v_lshlrev_b32 v{P.B0D[r]}, 1, v{P.B0[r]}" for r in range(M)])
    else:
        e.emit(f"v_lshlrev_b32 v{P.XD}, 1, v{P.X[0]}")
    for i in range(L):
        e.extend(cyc_row(g, P, i))
        if i == MID - 1:
            e.extend(cyc_mid_reduce(g, P, i + 1))
    e.extend(cyc_normalise_store(g, P))
    return rotate_carries(e.out, carries)


# ------------------------------------------------------------------------------------------
# The short-base product x h 2^-261 (tools/gen_nadic_asm.py's mul_short: rows = h's KS limbs,
# digit 1 of the multiplier 0, KS quotient digits) over a lane group: the multiplier rows are
# LDS rows HROW .. HROW + KS - 1 of the ciphertext's column (every lane of the group reads the
# same word: a broadcast, one row ahead, as the general product's rows), B = the lane's slice of
# X (its own column, undoubled), the t window from 0, the s window from the pairs (D_j, 0) of
# the lane's columns (D = N - 2^261; the triple's dummy lane reads zeros: its column stays 0),
# the retiring-column adds 2^29 - 1 - q_i (+ 1 in row 0) as literals.  KS rows of 4 M + 1
# multiplies per lane (triple: 49, quad: 37), no mid-product reduction (a column gathers at
# most KS rows of two products < 2^58).
# ------------------------------------------------------------------------------------------
KS = 9
HROW = 2 * L + 2   # LDS row of h's limb 0 (after the two digits and the two spare rows)


def mul_short(g, carries=CARRY_PAIRS):
    e = Emitter()
    XA, XB = g.XA, g.XB
    e.extend(load_b_lds(g, False))
    e.extend([f"ds_read_b64 {g.As(r)}, %[dl] offset:{8 * r}" for r in range(g.M - 1)] +
             [f"ds_read_b64 {g.RS}, %[dl] offset:{8 * (g.M - 1)}"])
    e.extend([f"v_mov_b32 {g.RTHI}, 0", f"v_mov_b32 {g.MASKV}, {MASK}",
              f"v_add_u32 {g.AADR}, {HROW * g.ROWB}, %[ac]", f"ds_read_b32 {XA[0]}, {g.AADR}",
              "s_waitcnt lgkmcnt(0)"])
    for i in range(KS):
        xs, xn = (XA, XB) if i % 2 == 0 else (XB, XA)
        e.extend(row(g, i == 0, True, hex(1 << LB) if i == 0 else MASK, xs, xn, g.ROWB, first_s=False))
        e.extend([f"v_add_u32 {g.AADR}, {g.ROWB}, {g.AADR}", "s_waitcnt lgkmcnt(0)"])
    e.extend(normalise_store(g))
    return rotate_carries(e.out, carries)


def ms_mads(g):
    return sum(1 for ln in mul_short(g) if ln.startswith("v_mad_u64_u32"))


def row_mads(sq, g=QUAD):
    return sum(1 for ln in row(g, False, sq, "s35", g.XA, g.XB, g.ROWB) if ln.startswith("v_mad_u64_u32"))


def product_mads(sq, g=QUAD):
    if sq and CYC_SQUARE:  # unrolled: the static count is the executed count
        return sum(1 for ln in square_cyc(g) if ln.startswith("v_mad_u64_u32"))
    return L * row_mads(sq, g) + sum(1 for ln in mid_reduce(g) if ln.startswith("v_mad_u64_u32"))


def clobbers(g):
    regs = [f'"v{i}"' for i in range(max(g.NREG, CycPlan(g).NREG))]
    regs += [f'"s{i}"' for i in [19, 20, 21, 34, 35, 36] + list(range(KBASE, KBASE + L))]
    out = [", ".join(regs[i:i + 16]) for i in range(0, len(regs), 16)]
    return " \\\n  ".join(x + "," for x in out[:-1]) + " \\\n  " + out[-1]


def c_string(lines):
    return "\n".join(f'  "{ln}\\n"' for ln in lines)


def header(g, pfx, PFX, name):
    M = g.M
    mm, sq, ms = product(False, g), product(True, g), mul_short(g)
    sql = product(True, g, cyc=False)
    operands = ", ".join([f'[n{r}] "v"(n[{r}])' for r in range(M)])
    bp_doc, bp_arg, bp_op = "", "", ""
    mq_def = ""
    if g.G == 3:
        bp_doc = ("\n// bp: ds_bpermute byte address of the group's lane 0 (4 * (3 * (lane / 3)), the dummy lane 63\n"
                  "// its own).")
        bp_arg = ", uint32_t bp"
        bp_op = ', [bp] "v"(bp)'
        if TRI_DPP_BCAST:  # the quotient digits' lane mask (see gen_quad_asm.TRI_DPP_BCAST)
            bp_op += ', [mq] "v"(mq)'
            mq_def = "  const uint32_t mq = e0 ? 0x1fffffffu : 0u;\n"
    dpp_word = "DPP quad_perm" if g.G == 4 else "ds_bpermute broadcasts, DPP wave shifts"
    return f"""// GENERATED by tools/gen_quad_asm.py -- do not edit by hand.
//
// gfx950 assembly N-adic Montgomery product modulo N^2 over a {name} of lanes ({g.G} lanes per
// ciphertext, lane l owns limbs {M} l .. {M} l + {M - 1} of both 36-limb digits, radix 2^29,
// R = 2^1044; {dpp_word}): the LDS column a <- a * b * R^-1 (mod N^2), digits lazily < 2N.
// See tools/gen_quad_asm.py for the layout, the cross-lane steps and the bounds.
// {len(mm)} instructions (general, B from global; a runtime row loop), {len(sq)} (square{", unrolled cyclic-band triangular" if CYC_SQUARE else ""});
// per lane {product_mads(False, g)} / {product_mads(True, g)} v_mad_u64_u32 per product ({row_mads(False, g)} per general row).
#pragma once
#include <stdint.h>

#define FBM_{PFX}_LB {LB}
#define FBM_{PFX}_L {L}
#define FBM_{PFX}_LIMBS {M}
#define FBM_{PFX}_ROWW {g.ROWW}
#define FBM_{PFX}_ROWB {g.ROWB}
#define FBM_{PFX}_D1 {g.D1}
#define FBM_{PFX}_MADS_MUL {product_mads(False, g)}
#define FBM_{PFX}_MADS_SQR {product_mads(True, g)}
#define FBM_{PFX}_MADS_SHORT {ms_mads(g)}
#define FBM_{PFX}_HROW {HROW}

#define FBM_{PFX}_CLOBBERS \\
  {clobbers(g)}

// n: the lane's {M} limbs of N (N_({M} l + r)); e0 = (lane is the group's lane 0); ac: LDS byte address
// of the ciphertext column (limb 0 of digit 0), al = ac + {M} l * ROWB; QK: the quad constants block
// (K'_i = 2^29 - 1 + K_i, K = (1 - R) mod N, at words 0..35); np = -N^-1 mod 2^29.{bp_doc}

// B from global memory, table layout: limb row j (b0: j = r, b1: j = {M} + r) at
// bb + b_off + j * 1024 (bytes; bb uniform, b_off the lane's offset).
__device__ __forceinline__ void fbm_{pfx}_mm_glb(uint32_t ac, uint32_t al, const uint32_t* bb, uint32_t b_off,
                                              const uint32_t* QK, uint32_t np, const uint32_t (&n)[{M}],
                                              uint32_t e0{bp_arg}) {{
{mq_def}  asm volatile(
{c_string(mm)}
      :
      : [ac] "v"(ac), [al] "v"(al), [b] "v"(b_off), [bb] "s"(bb), [QK] "s"(QK), [np] "s"(np), [e0] "v"(e0){bp_op},
        {operands}
      : "memory", "vcc", "scc", FBM_{PFX}_CLOBBERS);
}}

// a <- a h 2^-{LB * KS} (mod N^2), h < 2^{LB * KS} in LDS rows {HROW} .. {HROW + KS - 1} of the column (row {HROW + KS}:
// the last row's prefetch); dl: LDS byte address of the pairs (D_j, 0) of the lane's columns
// (D = N - 2^{LB * KS}; zeros for a dummy lane).  {len(ms)} instructions, {ms_mads(g)} v_mad_u64_u32 per lane.
__device__ __forceinline__ void fbm_{pfx}_ms_lds(uint32_t ac, uint32_t al, uint32_t dl, uint32_t np,
                                              const uint32_t (&n)[{M}], uint32_t e0{bp_arg}) {{
{mq_def}  asm volatile(
{c_string(ms)}
      :
      : [ac] "v"(ac), [al] "v"(al), [dl] "v"(dl), [np] "s"(np), [e0] "v"(e0){bp_op},
        {operands}
      : "memory", "vcc", "scc", FBM_{PFX}_CLOBBERS);
}}

// The looped square ({len(sql)} instructions): the table path's squares (small moduli, FDH retries -- cold), so
// the launch's hot code keeps one copy of the unrolled cyclic-band square.
__device__ __forceinline__ void fbm_{pfx}_sq_lds_looped(uint32_t ac, uint32_t al, const uint32_t* QK, uint32_t np,
                                                     const uint32_t (&n)[{M}], uint32_t e0{bp_arg}) {{
{mq_def}  asm volatile(
{c_string(sql)}
      :
      : [ac] "v"(ac), [al] "v"(al), [QK] "s"(QK), [np] "s"(np), [e0] "v"(e0){bp_op},
        {operands}
      : "memory", "vcc", "scc", FBM_{PFX}_CLOBBERS);
}}

// a <- a^2 R^-1 (mod N^2): B = A from the LDS column (the s part as x0 * (2 x1)).
__device__ __forceinline__ void fbm_{pfx}_sq_lds(uint32_t ac, uint32_t al, const uint32_t* QK, uint32_t np,
                                              const uint32_t (&n)[{M}], uint32_t e0{bp_arg}) {{
{mq_def}  asm volatile(
{c_string(sq)}
      :
      : [ac] "v"(ac), [al] "v"(al), [QK] "s"(QK), [np] "s"(np), [e0] "v"(e0){bp_op},
        {operands}
      : "memory", "vcc", "scc", FBM_{PFX}_CLOBBERS);
}}
""", mm, sq


# module-level names kept for tests/test_quad_asm.py (the quad geometry)
M, ROWW, ROWB, D1 = QUAD.M, QUAD.ROWW, QUAD.ROWB, QUAD.D1


def main():
    for g, pfx, PFX, name, fn in ((QUAD, "qa", "QA", "QUAD", "fbm_quad_asm.hpp"),
                                  (TRI, "ta", "TA", "TRIPLE", "fbm_tri_asm.hpp")):
        hdr, mm, sq = header(g, pfx, PFX, name)
        out = os.path.join(ROOT, "fedbiomed_amd", "csrc", fn)
        with open(out, "w") as f:
            f.write(hdr)
        print(f"wrote {out}: general {len(mm)} / square {len(sq)} instructions; mads/product {product_mads(False, g)} / "
              f"{product_mads(True, g)}; {max(g.NREG, CycPlan(g).NREG)} VGPRs")


if __name__ == "__main__":
    main()
