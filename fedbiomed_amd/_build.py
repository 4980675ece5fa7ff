"""Builds the in-tree gfx950 HIP library `fedbiomed_amd/_lib/libfbm_secagg.so` (and the
list API's host conversion module `_fbm_pyconv`, csrc/fbm_pyconv.c).

    python -m fedbiomed_amd._build            # incremental (rebuilds when a source is newer)
    python -m fedbiomed_amd._build --force

hipcc cross-compiles for gfx950 without a GPU.  -ffp-contract=off is load-bearing: the
quantise / average / dequantise FP64 sequences must round exactly like CPython + numpy.
"""

import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_lib", "libfbm_secagg.so")
SOURCES = ["fbm_lom.hip", "fbm_jl.hip", "fbm_gen.hip", "fbm_ass.hip", "fbm_capi.hip"]
# host-side list <-> buffer conversions of the list API (a CPython extension, plain gcc)
PYCONV_SRC = os.path.join(CSRC, "fbm_pyconv.c")
PYCONV_OUT = os.path.join(HERE, "_lib", "_fbm_pyconv" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
ARCH = os.environ.get("FBM_OFFLOAD_ARCH", "gfx950")
# a plain C99 caller of the C ABI (tests/test_c_client.py): the binding a non-Python host would write
CCLIENT_SRC = os.path.join(ROOT, "tests", "c_client", "fbm_c_roundtrip.c")
CCLIENT_OUT = os.path.join(ROOT, "tests", "c_client", "fbm_c_roundtrip")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp"))]
    inc = os.path.join(ROOT, "include")
    deps += [os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build_pyconv(force: bool = False, verbose: bool = False) -> str:
    if not force and os.path.exists(PYCONV_OUT) and os.path.getmtime(PYCONV_OUT) >= os.path.getmtime(PYCONV_SRC):
        return PYCONV_OUT
    os.makedirs(os.path.dirname(PYCONV_OUT), exist_ok=True)
    tmp = PYCONV_OUT + ".tmp"
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared", "-Wall", "-Werror",
           "-pthread", "-I" + sysconfig.get_paths()["include"], PYCONV_SRC, "-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, PYCONV_OUT)
    return PYCONV_OUT


def build_c_client(force: bool = False, verbose: bool = False) -> str:
    """gcc, C99, against include/fbm_secagg.h and the in-tree library (found through an $ORIGIN rpath,
    so the tree can move, as it does to the GPU box) plus the HIP runtime for its device buffers."""
    deps = [CCLIENT_SRC, OUT, os.path.join(ROOT, "include", "fbm_secagg.h")]
    if not force and os.path.exists(CCLIENT_OUT) and all(
            os.path.getmtime(CCLIENT_OUT) >= os.path.getmtime(d) for d in deps):
        return CCLIENT_OUT
    rel = os.path.relpath(os.path.dirname(OUT), os.path.dirname(CCLIENT_OUT))
    tmp = CCLIENT_OUT + ".tmp"
    cmd = [os.environ.get("CC", "gcc"), "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROCM, "include"), CCLIENT_SRC,
           "-L" + os.path.dirname(OUT), "-lfbm_secagg", "-L" + os.path.join(ROCM, "lib"), "-lamdhip64",
           "-Wl,-rpath,$ORIGIN/" + rel, "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, CCLIENT_OUT)
    return CCLIENT_OUT


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """`out` / `defines`: variant builds for A/B measurement (tools/ab.sh); the product is OUT.
    The host conversion module is optional: if it does not build (an interpreter whose headers
    it does not support), the list API uses its pure-Python conversions (_device._PyConvFallback)
    and the HIP library still builds."""
    if out == OUT and not defines:
        try:
            build_pyconv(force, verbose)
        except (subprocess.CalledProcessError, OSError) as e:
            print(f"warning: {PYCONV_SRC} did not build ({e}); the list API falls back to Python conversions")
    if out == OUT and not defines and not force and not needs_build():
        build_c_client(force, verbose)
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
           "-I" + os.path.join(ROOT, "include")] + ["-D" + d for d in defines] + \
        [os.path.join(CSRC, f) for f in SOURCES] + ["-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    if out == OUT and not defines:
        build_c_client(True, verbose)
    return out


if __name__ == "__main__":
    # python -m fedbiomed_amd._build [--force] [--out PATH] [-DNAME[=V] ...]
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else OUT
    defs = [a[2:] for a in args if a.startswith("-D")]
    print(build(force="--force" in args, verbose=True, out=out, defines=defs))
