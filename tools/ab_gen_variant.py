#!/usr/bin/env python3
"""Builds an A/B variant of the library whose generated assembly headers come from the generators
run under environment switches (e.g. FBM_GEN_TRI_DPP=1, tools/gen_quad_asm.py): the headers are
written into a copy of csrc/, never over the shipped ones.

    FBM_GEN_TRI_DPP=1 python tools/ab_gen_variant.py tridpp     # -> build/ab/tridpp.so

Load it with FBM_LIB_PATH=build/ab/<name>.so (tools/exp_probe.py, bench.py)."""

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


def main(name):
    work = f"/tmp/ab_gen_{name}"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work + "/x")
    shutil.copytree(B.CSRC, work + "/x/csrc")
    shutil.copytree(os.path.join(ROOT, "include"), work + "/include")
    for g, pfx, PFX, nm, fn in ((G.QUAD, "qa", "QA", "QUAD", "fbm_quad_asm.hpp"),
                                (G.TRI, "ta", "TA", "TRIPLE", "fbm_tri_asm.hpp")):
        hdr, _, _ = G.header(g, pfx, PFX, nm)
        with open(os.path.join(work, "x", "csrc", fn), "w") as f:
            f.write(hdr)
    out0 = NA.OUT
    NA.OUT = os.path.join(work, "x", "csrc", "fbm_nadic_asm.hpp")
    NA.main()
    NA.OUT = out0
    os.makedirs(os.path.join(ROOT, "build", "ab"), exist_ok=True)
    out = os.path.join(ROOT, "build", "ab", f"{name}.so")
    cmd = [B.hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
           f"-I{work}/include"] + [os.path.join(work, "x", "csrc", f) for f in B.SOURCES] + ["-o", out]
    return subprocess.call(cmd)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
