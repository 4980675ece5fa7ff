#!/usr/bin/env python3
"""Per-kernel resources of a built library, read from its gfx950 code objects (no GPU needed).

The shared library's .hip_fatbin section holds one clang offload bundle per translation unit; each
bundle's gfx950 entry is an ELF code object whose NT_AMDGPU_METADATA note lists every kernel's
VGPRs, AGPRs, SGPRs, scratch bytes per lane (private_segment_fixed_size), LDS bytes per workgroup
(group_segment_fixed_size) and maximum workgroup size.  Waves per SIMD by registers: gfx950 has 512
unified registers per lane; the metadata's vgpr_count is the unified total (AGPRs included: a kernel past
256 architectural VGPRs spills into AGPRs), allocated in granules of 8.

    python tools/kernel_resources.py [fedbiomed_amd/_lib/libfbm_secagg.so] [--json out.json]

Used by tests/test_kernel_resources.py (the combine kernels' zero scratch and two waves per SIMD).
"""
import json
import os
import shutil
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "fedbiomed_amd", "_lib", "libfbm_secagg.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(lib_path, arch="gfx950"):
    """The `arch` code objects of every offload bundle in the library (bytes each)."""
    with open(lib_path, "rb") as f:
        data = f.read()
    objs, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return objs
        off = i + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, off)
        off += 8
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if triple.endswith(arch) and es:
                objs.append(data[i + eo:i + eo + es])
        pos = i + len(MAGIC)


def _align(v, g=8):
    return (v + g - 1) // g * g


def kernels(lib_path=DEFAULT_LIB, arch="gfx950"):
    """{demangled kernel name: resources} over every code object of the library."""
    import yaml

    out = {}
    with tempfile.TemporaryDirectory(prefix="fbm_kres_") as tmp:
        for j, obj in enumerate(code_objects(lib_path, arch)):
            p = os.path.join(tmp, f"co{j}.elf")
            with open(p, "wb") as f:
                f.write(obj)
            notes = subprocess.run([READELF, "--notes", p], capture_output=True, text=True, check=True).stdout
            start = notes.index("---")
            end = notes.index("...", start)
            meta = yaml.safe_load(notes[start:end])
            for k in meta.get("amdhsa.kernels", []):
                v, a = k.get(".vgpr_count", 0), k.get(".agpr_count", 0)
                out[k[".name"]] = {
                    "vgpr": v, "agpr": a, "sgpr": k.get(".sgpr_count", 0),
                    "scratch_bytes_per_lane": k.get(".private_segment_fixed_size", 0),
                    "lds_bytes_per_workgroup": k.get(".group_segment_fixed_size", 0),
                    "max_workgroup_size": k.get(".max_flat_workgroup_size", 0),
                    "vgpr_spill": k.get(".vgpr_spill_count", 0), "sgpr_spill": k.get(".sgpr_spill_count", 0),
                    "dynamic_stack": bool(k.get(".uses_dynamic_stack", False)),
                    "waves_per_simd_by_registers": min(8, 512 // max(8, _align(v))),
                }
    cxxfilt = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    if out and cxxfilt:  # (without a demangler the names stay mangled; find() then matches a substring)
        names = list(out)
        dem = subprocess.run([cxxfilt], input="\n".join(names), capture_output=True, text=True,
                             check=True).stdout.split("\n")
        out = {d.strip() or n: out[n] for n, d in zip(names, dem)}
    return out


def find(res, kernel):
    """The entries of `kernel` (e.g. "jl_prod_kernel"): every instantiation, demangled or not."""
    return {k: v for k, v in res.items() if f"fbm::{kernel}(" in k or f"fbm::{kernel}<" in k
            or f"{len(kernel)}{kernel}E" in k or f"{len(kernel)}{kernel}I" in k}


def main():
    args = sys.argv[1:]
    dst = None
    if "--json" in args:
        i = args.index("--json")
        dst = args[i + 1]
        del args[i:i + 2]
    res = kernels(args[0] if args else DEFAULT_LIB)
    for name in sorted(res):
        r = res[name]
        print(f"{name[:90]:90s} vgpr {r['vgpr']:3d} agpr {r['agpr']:3d} scratch {r['scratch_bytes_per_lane']:5d} "
              f"lds {r['lds_bytes_per_workgroup']:6d} waves/SIMD(regs) {r['waves_per_simd_by_registers']}")
    if dst:
        with open(dst, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
