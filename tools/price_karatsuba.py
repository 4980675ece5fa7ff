#!/usr/bin/env python3
"""Pricing of limb-level Karatsuba inside the JL exponentiation's square (round-5 VERDICT item 4: "split x0 x1,
the 36 x 36-limb cross product of the N-adic square, into 18-limb halves ... Gate: >= 4 % fewer issue slots per
square at <= 236 VGPRs.  Do the same count for the triple engine's square").  Counts only -- nothing is built
unless it passes.  Writes profiles/r6_karatsuba_pricing.json.

The square: X = x0 + x1 N mod N^2, X^2 R^-1 = t + N s with t = REDC_N(x0^2) and
s = REDC_N(2 x0 x1 - m).  Both REDCs run row by row in one loop: row i multiplies the row operand (x0_i, doubled)
into a 36-column window of 64-bit accumulators per part and retires the window's lowest column (its quotient
digit q_i / q'_i times N).  Column j must hold every product of x0 x1 that lands in it when row j retires it.

Karatsuba on x0 x1 (a = x0 = a0 + a1 B, b = x1 = b0 + b1 B, B = 2^(29*18)):
    a b = z0 (1 - B) + z1' B + z2 (B^2 - B),   z0 = a0 b0, z2 = a1 b1, z1' = (a0 + a1)(b0 + b1)
saves 1296 - 3 * 324 = 324 of the 1296 cross-product multiplies -- IF z0's and z2's column sums are formed once
and added at two positions each (c and c + 18; c + 18 and c + 36).  Three ways to place them in the row-scanned
REDC, each counted here instruction class by instruction class:

  dup     no column sums: every z0 / z2 product multiplied twice (the second one signed, into column c + 18)
          and z1' in the same rows.  A row then reaches columns i .. i + 53: the window grows by 18 pairs.
  vgpr    column sums materialised: z0, z1', z2 product-scanned (column by column, in the REDC's order) into
          temporaries; z0_c and z2_c are needed again 18 rows later, so 18 + 18 pending 64-bit sums stay in
          VGPRs, with the half sums (a0 + a1), (b0 + b1) (18 + 18 VGPRs).
  lds     the same with the pending column sums in LDS (one 64-bit write and read each), the half sums in VGPRs.

Issue costs per wave-instruction at two waves per SIMD (tools/microbench/gen_oprate.py): a
v_mad_u64_u32 3.8-4.4 SIMD clocks (4.1 taken), a 64-bit shift / add 3.5, v_mul_lo_u32 and DPP 3.4, a 32-bit op
2.25, an LDS instruction 1 (its bandwidth is checked separately).  Column bounds by interval arithmetic on the
operand bounds (29-bit limbs, 30-bit half sums).

    python tools/price_karatsuba.py
"""

import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_nadic_asm as GN  # noqa: E402
import gen_quad_asm as GQ  # noqa: E402

COST = {"mad": 4.1, "valu64": 3.5, "mul_lo": 3.4, "dpp": 3.4, "valu32": 2.25, "lds": 1.0, "salu": 0.0}
VGPR_GATE, SLOT_GATE = 236, 0.04
COMPILER_VGPRS = 6  # the kernel around the square: 236 VGPRs in all with the square's 230 (ISA, r4)
TRI_KERNEL_VGPRS = 168  # jl_expg_kernel<3>: 3 waves per SIMD (profiles/archive/r4_kernel_resources.txt)


def classify(ln):
    op = ln.split()[0]
    if op in ("v_mad_u64_u32", "v_mad_i64_i32"):
        return "mad"
    if op == "v_mul_lo_u32":
        return "mul_lo"
    if "_dpp" in op or op in ("ds_bpermute_b32", "v_mov_b32_dpp"):
        return "dpp"
    if op in ("v_lshrrev_b64", "v_lshl_add_u64", "v_lshlrev_b64"):
        return "valu64"
    if op.startswith("v_"):
        return "valu32"
    if op.startswith("ds_"):
        return "lds"
    return "salu"


def clocks(counts):
    return sum(COST[k] * v for k, v in counts.items())


def column_bound(terms, a_bits, b_bits):
    """Upper bound of a column holding `terms` products of an a_bits-bit and a b_bits-bit limb."""
    return terms * ((1 << a_bits) - 1) * ((1 << b_bits) - 1)


def one_lane():
    lines = GN.square_unrolled()
    shipped = collections.Counter(classify(ln) for ln in lines)
    L, H = GN.L, GN.L // 2
    cross = sum(1 for ln in lines if ln.startswith("v_mad_u64_u32")
                and any(f" {GN.SB1(j)}," in ln for j in range(L)))
    assert cross == L * L
    base_clk = clocks(shipped)
    vgprs = GN.SQ_NREG + COMPILER_VGPRS
    sub = 3 * H * H  # the three half products
    out = {"shipped": {"counts": dict(shipped), "issue_clocks": base_clk, "vgprs": vgprs,
                       "cross_product_mads": cross},
           "ideal": {"mads_saved": cross - sub, "issue_clocks_saved": COST["mad"] * (cross - sub),
                     "frac_of_square": COST["mad"] * (cross - sub) / base_clk,
                     "note": "multiplies only, every other cost zero: the ceiling of any Karatsuba layout"}}
    # column bounds: z1' columns hold up to 18 products of two 30-bit half sums
    b_z1 = column_bound(H, LB + 1, LB + 1)
    b_z0 = column_bound(H, LB, LB)
    out["bounds"] = {"z1_column_max_log2": b_z1.bit_length(), "z1_fits_64": b_z1 < 1 << 64,
                     "z0_column_max_log2": b_z0.bit_length(), "z0_fits_64": b_z0 < 1 << 64,
                     "note": "18 products of (2^30 - 1)^2 pass 2^64: z1' needs two accumulators per column (or a "
                             "mid pass); z0 / z2 columns of 18 products of 29-bit limbs fit"}
    variants = {}
    # dup: rows i < 18 (operand a0_i, a1_i, a0_i + a1_i) -- z0 + (-z0) + z1' + (-z2) + z2: 5 x 18 mads a row
    d = collections.Counter(shipped)
    d["mad"] += H * 5 * H - cross
    d["valu32"] += H + H + 2 * H  # u_i per row, v_k once, -a0_i / -a1_i per row
    d["valu64"] += 0
    variants["dup"] = {"counts": dict(d), "vgprs": vgprs + H + 2 * H,
                       "extra_vgprs": {"v = b0 + b1": H, "s window 36 -> 54 columns": 2 * H},
                       "note": "a row of 18-limb halves reaches columns i .. i + 53 (the window grows by 18 pairs); "
                               "every z0 / z2 product is multiplied twice (the second, signed, into column + 18)"}
    # vgpr / lds: product-scanned column sums, recombined into the s window at the REDC's pace
    ncol = 2 * H - 1  # 35 columns per half product
    rec = collections.Counter()
    rec["mad"] = sub - cross                       # 972 multiplies instead of 1296
    rec["valu32"] += 2 * H                         # the half sums a0 + a1, b0 + b1 (once per square)
    rec["valu64"] += ncol * 2                      # z0, z2: the second product-scan accumulator folded in
    rec["valu64"] += ncol * 2                      # z1': two accumulators (bounds), folded, then += 2 z1' at c + 18
    rec["valu64"] += 2 * ncol                      # z0_c: += 2 z0_c at c; z2_c: += 2 z2_c at c + 36 (v_lshl_add)
    rec["valu64"] += 2 * ncol                      # z0_c, z2_c: shifted by 1 for the subtraction at c + 18
    rec["valu32"] += 2 * 2 * ncol                  # ... and subtracted (sub_co + subb_co)
    v = collections.Counter(shipped)
    v.update(rec)
    variants["vgpr"] = {"counts": dict(v), "vgprs": vgprs + 2 * H + 2 * 2 * H + 8,
                        "extra_vgprs": {"half sums": 2 * H, "pending z0_c, z2_c (18 + 18 pairs)": 4 * H,
                                        "product-scan accumulators": 8}}
    ldsv = collections.Counter(v)
    ldsv["lds"] += 2 * 2 * H                       # pending sums: one 64-bit write and one read each (z0, z2)
    variants["lds"] = {"counts": dict(ldsv), "vgprs": vgprs + 2 * H + 8,
                       "extra_vgprs": {"half sums": 2 * H, "product-scan accumulators": 8},
                       "lds_bytes_per_lane": 2 * H * 8}
    for k, var in variants.items():
        c = var["counts"]
        var["issue_clocks"] = clocks(c)
        var["slot_change"] = (var["issue_clocks"] - base_clk) / base_clk
        var["mads"] = c["mad"]
        var["passes_gate"] = var["slot_change"] <= -SLOT_GATE and var["vgprs"] <= VGPR_GATE
    out["variants"] = variants
    return out


LB = GN.LB


def triple():
    g = GQ.TRI
    P = GQ.CycPlan(g)
    lines = GQ.square_cyc(g)
    shipped = collections.Counter(classify(ln) for ln in lines)
    b1 = {f"v{r}" for r in P.B1}
    cross = sum(1 for ln in lines if ln.startswith("v_mad_u64_u32")
                and any(x.strip() in b1 for x in ln.split(",")[2:4]))
    L, M, H = GN.L, g.M, GN.L // 2
    assert cross == L * M, cross
    base_clk = clocks(shipped)
    vg = TRI_KERNEL_VGPRS  # the square's plan (P.NREG) plus what the kernel keeps live around it
    # per lane: the 36 x 12 cross products become 3 half products over the lane's share: 972 / 3 = 324 a lane
    saved = cross - 3 * H * H // g.G
    out = {"shipped": {"counts": dict(shipped), "issue_clocks": base_clk, "vgprs": vg, "cross_product_mads": cross,
                       "waves_per_simd": 512 // vg},
           "ideal": {"mads_saved_per_lane": saved, "frac_of_square": COST["mad"] * saved / base_clk}}
    # the halves straddle lanes (limbs 0-11 | 12-23 | 24-35 per lane, halves 0-17 | 18-35): the half sums b0 + b1
    # of a lane's limbs need the partner limb 18 away -- on another lane (DPP / bpermute, then add), and z0 / z2's
    # second position (column + 18) lies 1.5 lanes away in the band: every pending column sum crosses lanes
    r = collections.Counter(shipped)
    r["mad"] -= saved
    r["dpp"] += M                   # partner limbs of b for the half sums (once per square)
    r["valu32"] += M + H            # b half sums; a half sums per row (rows < 18)
    r["dpp"] += 2 * 2 * (2 * H - 1) // g.G       # pending z0 / z2 sums moved to the lane 18 columns up (lo, hi)
    r["valu64"] += 3 * 2 * (2 * H - 1) // g.G    # the three half products' column sums folded in (lshl_add)
    r["valu32"] += 2 * 2 * (2 * H - 1) // g.G    # and the two subtractions at column + 18 (sub_co + subb_co)
    extra = M + 4 * H // g.G + 4    # b half sums, this lane's pending sums, scan accumulators
    v = vg + extra
    var = {"counts": dict(r), "issue_clocks": clocks(r), "vgprs": v, "waves_per_simd": 512 // v,
           "note": "the triple runs 3 waves per SIMD at <= 170 VGPRs; past it 2 (w = 2 -> 3 measured 5.64 -> 5.48 us "
                   "per square per wave, profiles/archive/r3_carry_rotation_ab.jsonl)"}
    var["slot_change"] = (var["issue_clocks"] - base_clk) / base_clk
    var["passes_gate"] = var["slot_change"] <= -SLOT_GATE and var["waves_per_simd"] >= out["shipped"]["waves_per_simd"]
    out["variants"] = {"column_sums": var}
    return out


def main():
    res = {"meta": {"tool": "tools/price_karatsuba.py", "costs_clocks_per_wave_instruction_at_2_waves": COST,
                    "gate": f">= {100 * SLOT_GATE:.0f} % fewer issue clocks per square at <= {VGPR_GATE} VGPRs "
                            "(the triple: without losing its third wave per SIMD)",
                    "reference": "/root/reference/fedbiomed/common/secagg/_jls.py:60-73 (powmod), 473-505 (encrypt)"},
           "one_lane": one_lane(), "triple": triple()}
    ok = [f"one_lane.{k}" for k, v in res["one_lane"]["variants"].items() if v["passes_gate"]]
    ok += [f"triple.{k}" for k, v in res["triple"]["variants"].items() if v["passes_gate"]]
    res["verdict"] = {"build": ok, "decision": "build " + ", ".join(ok) if ok else
                      "no-go: no layout passes the gate -- not built"}
    path = os.path.join(ROOT, "profiles", "r6_karatsuba_pricing.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    o = res["one_lane"]
    print(f"one-lane square: {o['shipped']['issue_clocks']:.0f} clocks, {o['shipped']['vgprs']} VGPRs; ideal saving "
          f"{100 * o['ideal']['frac_of_square']:.1f} %")
    for k, v in o["variants"].items():
        print(f"  {k:5s} mads {v['mads']:5d}  slots {100 * v['slot_change']:+6.1f} %  VGPRs {v['vgprs']}  "
              f"gate {'PASS' if v['passes_gate'] else 'fail'}")
    t = res["triple"]
    print(f"triple square: {t['shipped']['issue_clocks']:.0f} clocks, {t['shipped']['vgprs']} VGPRs; ideal "
          f"{100 * t['ideal']['frac_of_square']:.1f} %")
    for k, v in t["variants"].items():
        print(f"  {k}: slots {100 * v['slot_change']:+6.1f} %  VGPRs {v['vgprs']} ({v['waves_per_simd']} waves)  "
              f"gate {'PASS' if v['passes_gate'] else 'fail'}")
    print(res["verdict"]["decision"])


if __name__ == "__main__":
    main()
