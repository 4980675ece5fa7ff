#!/usr/bin/env python3
"""Instruction-count pricing of triple-engine square layouts (round-5 VERDICT item 2: "price DESIGN.md:943-945's
layout on the simulator first; build it only if the instruction count drops >= 10 % per square").

Counts, per row of the cyclic-band square (36 rows, tools/gen_quad_asm.py) and per square, the VALU instructions
of one lane of a group -- the wave's issue count, every lane running the same stream:

* shipped      -- the generator's own rows (cyc_row(TRI, ...)), classified instruction by instruction: the
                  t / s products, the q N / q' N products, the quotient chain (mul_lo, and, K' - q, the e0
                  mad), the two retires (and_dpp hand-down, 64-bit shift, 64-bit add);
* fixed_column -- column c owned by lane c mod 3 for its whole life (the retiring column never changes lanes, so
                  the K' fold applies: one signed mad q * E_i per row instead of K' - q and the e0 mad); each
                  lane needs all 36 limbs of b0, 2 b1 and N (the column of x_i * b_k is (i + k) mod 3), the t
                  products are the triangle's 36 - i per row over three lanes, and each retire moves the
                  retiring column's 35-bit carry to the next lane: 64-bit shift, the carry masked to the owning
                  lane (2), two DPP moves, one 64-bit add;
* unmasked_down -- the shipped layout, with lanes 1-2 handing their low dword down unmasked and carrying hi * 8
                  (one mad), and lane 0 -- whose bits 29-31 the lane below must not receive -- adding them with a
                  second masked mad after a 32-bit shift: per part 1 DPP + 3 instead of 1 DPP + 2.
The row counts of the alternatives are written out from their per-row instruction lists below (the same classes
as the shipped rows); the shipped count is the generator's.  Writes profiles/archive/r5_tri_layout_pricing.json.

    python tools/price_tri_layouts.py
"""

import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_quad_asm as G  # noqa: E402


def classify(ln, P):
    op = ln.split()[0]
    if not op.startswith("v_"):
        return None
    if op == "v_mad_u64_u32":
        srcs = [x.strip() for x in ln.split(",")]
        if "%[e0]" in ln:
            return "chain"          # (K'_i - q) * e0 into the s window
        return "mad"
    if op in ("v_mul_lo_u32", "v_and_b32", "v_sub_u32"):
        return "chain"
    if op.startswith("v_and_b32_dpp") or op in ("v_lshrrev_b64", "v_lshl_add_u64"):
        return "retire"
    return "other"


def shipped_rows():
    P = G.CycPlan(G.TRI)
    rows = []
    for i in range(G.L):
        c = collections.Counter()
        for ln in G.cyc_row(G.TRI, P, i):
            k = classify(ln, P)
            if k:
                c[k] += 1
        rows.append(dict(c))
    return rows


def fixed_column_rows():
    """Per-row lists of the fixed-column layout (see the docstring)."""
    rows = []
    for i in range(G.L):
        t_prod = -(-(G.L - i) // 3)  # the triangle's 36 - i products of row i over three lanes (busiest lane)
        mads = t_prod + 12 + 12 + 12  # t, s (x_i * 2 x1 over the lane's 12 columns), q N, q' N
        chain = 2 + 1 + 2             # q: mul_lo + and; the folded subtraction: v_mad_i64_i32 q * E_i; q': mul_lo + and
        retire = 2 * (1 + 2 + 2 + 1)  # per part: shift, mask to the owner (lo, hi), 2 DPP moves, 64-bit add
        rows.append({"mad": mads, "chain": chain, "retire": retire})
    return rows


def unmasked_down_rows(shipped):
    rows = []
    for r in shipped:
        r = dict(r)
        r["retire"] = 2 * (1 + 3)  # per part: DPP hand-down; hi * 8 mad, lo >> 29, masked mad (lane 0)
        rows.append(r)
    return rows


def total(rows):
    return {k: sum(r.get(k, 0) for r in rows) for k in ("mad", "chain", "retire", "other")}


def main():
    sh = shipped_rows()
    alts = {"shipped": sh, "fixed_column": fixed_column_rows(), "unmasked_down": unmasked_down_rows(sh)}
    base = sum(total(sh).values())
    out = {"meta": {"source": "tools/price_tri_layouts.py (round 5)", "engine": "triple (G = 3, M = 12), cyclic-band "
                    "square rows only (the square's prologue / normalisation are common to all three)",
                    "gate": "VERDICT r4 item 2: build only if the count drops >= 10 % per square"}, "layouts": {}}
    for name, rows in alts.items():
        t = total(rows)
        n = sum(t.values())
        out["layouts"][name] = {"per_square": t, "valu_per_square": n, "vs_shipped": round(n / base - 1, 4),
                                "row0": rows[0], "row35": rows[-1]}
        print(f"{name:14s} {n:6d} VALU per square ({n / base - 1:+.1%})  {t}")
    with open(os.path.join(ROOT, "profiles", "r5_tri_layout_pricing.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
