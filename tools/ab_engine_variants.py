#!/usr/bin/env python3
"""Library variants whose exponentiation-engine SQUARE keeps only its multiplies (plus the LDS
address arithmetic and the scalar control flow): garbage results, timing only -- the share of a
real launch that the square's other instructions cost (tools/exp_probe.py on the variant).

    python tools/ab_engine_variants.py tri nadic    # build/ab/{tri,nadic}_madsonly.so"""

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import gen_nadic_asm as NA  # noqa: E402
import gen_quad_asm as G  # noqa: E402
from fedbiomed_amd import _build as B  # noqa: E402


def madsonly(lines, addr_regs):
    def keep(ln):
        if not ln.startswith("v_"):
            return True
        if ln.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
            return True
        if ln.startswith(("v_add_u32 ", "v_mov_b32 ")):
            return ln.split()[1].rstrip(",") in addr_regs
        return False
    return [ln for ln in lines if keep(ln) and not ln.startswith("ds_bpermute")]


def build(engine):
    work = f"/tmp/ab_{engine}_madsonly"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work + "/x")
    shutil.copytree(B.CSRC, work + "/x/csrc")
    shutil.copytree(os.path.join(ROOT, "include"), work + "/include")
    if engine == "tri":
        orig = G.product

        def product(sq, g=G.QUAD, carries=G.CARRY_PAIRS, cyc=None):
            lines = orig(sq, g, carries, cyc)
            return madsonly(lines, {G.TRI.AADR}) if (sq and g is G.TRI and cyc is not False) else lines

        G.product = product
        hdr, _, _ = G.header(G.TRI, "ta", "TA", "TRIPLE")
        G.product = orig
        with open(work + "/x/csrc/fbm_tri_asm.hpp", "w") as f:
            f.write(hdr)
    else:
        orig, orig_u, out0 = NA.square_tri, NA.square_unrolled, NA.OUT
        NA.square_tri = lambda: madsonly(orig(), {NA.SAADR, NA.SDADDR, NA.STMP})  # (the looped square)
        NA.square_unrolled = lambda: madsonly(orig_u(), {NA.SAADR, NA.SDADDR, NA.STMP})  # the shipped square
        NA.OUT = work + "/x/csrc/fbm_nadic_asm.hpp"
        NA.main()
        NA.square_tri, NA.square_unrolled, NA.OUT = orig, orig_u, out0
    os.makedirs(os.path.join(ROOT, "build", "ab"), exist_ok=True)
    out = os.path.join(ROOT, "build", "ab", f"{engine}_madsonly.so")
    cmd = [B.hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
           f"-I{work}/include"] + [os.path.join(work, "x", "csrc", f) for f in B.SOURCES] + ["-o", out]
    return subprocess.Popen(cmd)


if __name__ == "__main__":
    procs = [build(e) for e in (sys.argv[1:] or ["tri", "nadic"])]
    print([p.wait() for p in procs])
