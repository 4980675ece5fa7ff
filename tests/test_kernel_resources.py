"""The shipped library's kernel resources, read from its gfx950 code objects (tools/kernel_resources.py; CPU
only).  Pins what DESIGN.md states about registers, scratch and LDS, so a compiler or source change that
spills a hot kernel, or pushes it to fewer waves per SIMD, fails here before it reaches a GPU:
  * the combine kernels (jl_prod_kernel, jl_encf_kernel): no scratch, <= 256 registers and <= 80 KB of LDS
    per workgroup -- two waves per SIMD;
  * the one-lane exponentiation (jl_exp_kernel): two waves per SIMD, its main loop's spill-free prologue
    budget (<= 104 B per lane) unchanged;
  * jl_lift_kernel and every HBM-bound LOM / ASS kernel: no scratch;
  * no kernel with a dynamic stack.
"""

import importlib.util
import os
import shutil

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fedbiomed_amd", "_lib", "libfbm_secagg.so")


@pytest.fixture(scope="module")
def res():
    spec = importlib.util.spec_from_file_location("kernel_resources", os.path.join(ROOT, "tools", "kernel_resources.py"))
    kr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(kr)
    if not os.path.exists(LIB):
        pytest.skip("library not built (python -m fedbiomed_amd._build)")
    if not os.path.exists(kr.READELF):
        pytest.skip("llvm-readelf not found")
    r = kr.kernels(LIB)
    assert r, "no gfx950 kernel metadata found in the library"
    return kr, r


def _one(kr, r, name):
    hits = kr.find(r, name)
    assert hits, f"{name} not in the library"
    return hits


@pytest.mark.parametrize("name", ["jl_prod_kernel", "jl_encf_kernel"])
def test_combine_kernels_two_waves_no_scratch(res, name):
    kr, r = res
    for k, v in _one(kr, r, name).items():
        assert v["scratch_bytes_per_lane"] == 0, (k, v)
        assert v["vgpr"] <= 256 and v["waves_per_simd_by_registers"] >= 2, (k, v)
        assert v["lds_bytes_per_workgroup"] <= 80 * 1024, (k, v)  # two workgroups in a CU's 160 KB


def test_exp_kernel_two_waves(res):
    kr, r = res
    for k, v in _one(kr, r, "jl_exp_kernel").items():
        assert v["waves_per_simd_by_registers"] >= 2, (k, v)
        assert v["lds_bytes_per_workgroup"] <= 80 * 1024, (k, v)
        assert v["scratch_bytes_per_lane"] <= 104, (k, v)


@pytest.mark.parametrize("name", ["jl_lift_kernel", "lom_protect_kernel", "lom_aggregate_kernel",
                                  "lom_aggregate_ws_kernel", "ass_split_kernel", "ass_reconstruct_kernel",
                                  "ass_reconstruct_ws_kernel", "jl_pack_kernel", "jl_decode_kernel",
                                  "jl_nude_kernel", "jl_fdh_kernel"])
def test_streaming_kernels_no_scratch(res, name):
    kr, r = res
    for k, v in _one(kr, r, name).items():
        assert v["scratch_bytes_per_lane"] == 0, (k, v)


def test_no_dynamic_stack(res):
    _, r = res
    assert not [k for k, v in r.items() if v["dynamic_stack"]]


def test_demangled_when_a_demangler_exists(res):
    _, r = res
    if shutil.which("c++filt") or shutil.which("llvm-cxxfilt"):
        assert any(k.startswith("fbm::") or "fbm::" in k for k in r)
