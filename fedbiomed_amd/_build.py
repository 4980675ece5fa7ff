"""Builds the in-tree gfx950 HIP libraries (and the list API's host conversion module
`_fbm_pyconv`, csrc/fbm_pyconv.c):

  fedbiomed_amd/_lib/libfbm_secagg.so       the product: exports exactly include/fbm_secagg.h
  fedbiomed_amd/_lib/libfbm_secagg_test.so  the test build: + include/fbm_secagg_test.h (host runs of
                                            device routines, per-thread engine switches, the per-kernel
                                            event timer) -- for tests/ and bench.py

Both link the SAME kernel objects (fbm_lom / fbm_jl / fbm_gen / fbm_ass, compiled once); only the
host-side C ABI (fbm_capi.hip) is compiled twice, the second time with -DFBM_TEST_HOOKS.  A linker
version script made from each library's header(s) keeps every other symbol local.

    python -m fedbiomed_amd._build            # incremental (rebuilds when a source is newer)
    python -m fedbiomed_amd._build --force

hipcc cross-compiles for gfx950 without a GPU.  -ffp-contract=off is load-bearing: the
quantise / average / dequantise FP64 sequences must round exactly like CPython + numpy.
"""

import os
import re
import subprocess
import sys
import sysconfig
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_lib", "libfbm_secagg.so")
TEST_OUT = os.path.join(HERE, "_lib", "libfbm_secagg_test.so")
KERNEL_SOURCES = ["fbm_lom.hip", "fbm_jl.hip", "fbm_gen.hip", "fbm_ass.hip"]
CAPI_SOURCE = "fbm_capi.hip"
SOURCES = KERNEL_SOURCES + [CAPI_SOURCE]
HEADER = os.path.join(ROOT, "include", "fbm_secagg.h")
TEST_HEADER = os.path.join(ROOT, "include", "fbm_secagg_test.h")
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


def declared(*headers) -> list:
    """The fbm_* functions the header(s) declare (a declaration starts at a line's beginning)."""
    names = []
    for h in headers:
        with open(h) as fh:
            for m in re.finditer(r"^[A-Za-z_][\w \t\*]*?\b(fbm_\w+)\s*\(", fh.read(), re.M):
                if m.group(1) not in names:
                    names.append(m.group(1))
    return names


def needs_build() -> bool:
    if not (os.path.exists(OUT) and os.path.exists(TEST_OUT)):
        return True
    t = min(os.path.getmtime(OUT), os.path.getmtime(TEST_OUT))
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


def _try_c_client(force: bool, verbose: bool) -> None:
    """The C client is test tooling: a box without gcc or the ROCm headers still gets the libraries."""
    try:
        build_c_client(force, verbose)
    except (subprocess.CalledProcessError, OSError) as e:
        print(f"warning: the C client {CCLIENT_SRC} did not build ({e}); tests/test_c_client.py will skip")


def _version_script(path: str, names) -> str:
    with open(path, "w") as fh:
        fh.write("{\n  global:\n" + "".join(f"    {n};\n" for n in names) + "  local:\n    *;\n};\n")
    return path


def _compile_all(jobs, verbose: bool) -> None:
    """jobs: [(cmd, what)], run in parallel (at most FBM_BUILD_JOBS / 8 at once); raises on the first failure."""
    width = max(1, int(os.environ.get("FBM_BUILD_JOBS", "8")))
    pending, running = list(jobs), []
    while pending or running:
        while pending and len(running) < width:
            cmd, what = pending.pop(0)
            if verbose:
                print(" ".join(cmd))
            running.append((subprocess.Popen(cmd), what, cmd))
        p, what, cmd = running.pop(0)
        if p.wait() != 0:
            for q, _, _ in running:
                q.kill()
                q.wait()
            raise subprocess.CalledProcessError(p.returncode, cmd)


def _build_libs(targets, defines, verbose: bool) -> None:
    """targets: [(out, test_hooks)] linked from one set of kernel objects."""
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
            "-I" + os.path.join(ROOT, "include")] + ["-D" + d for d in defines]
    with tempfile.TemporaryDirectory(prefix="fbm_build_") as tmpd:
        jobs, kobjs = [], []
        for f in KERNEL_SOURCES:
            o = os.path.join(tmpd, f.replace(".hip", ".o"))
            kobjs.append(o)
            jobs.append((base + ["-c", os.path.join(CSRC, f), "-o", o], f))
        capi = {}
        for test in sorted({t for _, t in targets}):
            o = os.path.join(tmpd, "fbm_capi_test.o" if test else "fbm_capi.o")
            capi[test] = o
            jobs.append((base + (["-DFBM_TEST_HOOKS"] if test else []) + ["-c", os.path.join(CSRC, CAPI_SOURCE),
                                                                         "-o", o], CAPI_SOURCE))
        _compile_all(jobs, verbose)
        for out, test in targets:
            names = declared(HEADER, TEST_HEADER) if test else declared(HEADER)
            vs = _version_script(os.path.join(tmpd, os.path.basename(out) + ".map"), names)
            os.makedirs(os.path.dirname(out), exist_ok=True)
            tmp = out + ".tmp"
            cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,--version-script=" + vs] + kobjs + \
                [capi[test], "-o", tmp]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
            os.replace(tmp, out)


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """The product library OUT and the test build TEST_OUT.  `out` / `defines`: a variant for A/B
    measurement (tools/ab.sh) -- one library at `out` with the test build's exports (the bench's
    timer) and -DFBM_AB_KNOBS (the A/B environment knobs) besides `defines`.
    The host conversion module is optional: if it does not build (an interpreter whose headers
    it does not support), the list API uses its pure-Python conversions (_device._PyConvFallback)
    and the HIP libraries still build."""
    variant = out != OUT or bool(defines)
    if not variant:
        try:
            build_pyconv(force, verbose)
        except (subprocess.CalledProcessError, OSError) as e:
            print(f"warning: {PYCONV_SRC} did not build ({e}); the list API falls back to Python conversions")
    if not variant and not force and not needs_build():
        _try_c_client(False, verbose)
        return OUT
    if variant:
        _build_libs([(out, True)], list(defines) + ["FBM_AB_KNOBS"], verbose)
        return out
    _build_libs([(OUT, False), (TEST_OUT, True)], [], verbose)
    _try_c_client(True, verbose)
    return OUT


if __name__ == "__main__":
    # python -m fedbiomed_amd._build [--force] [--out PATH] [-DNAME[=V] ...]
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else OUT
    defs = [a[2:] for a in args if a.startswith("-D")]
    print(build(force="--force" in args, verbose=True, out=out, defines=defs))
