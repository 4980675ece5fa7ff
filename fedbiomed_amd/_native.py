"""ctypes binding of the C-ABI HIP library (include/fbm_secagg.h).

The library is built in-tree (`python -m fedbiomed_amd._build` or
`__graft_entry__.build()`) to `fedbiomed_amd/_lib/libfbm_secagg.so`.  There is NO
CPU fallback: if the library or a GPU is missing, every compute call raises.

`load()` is the product library.  The test build `libfbm_secagg_test.so` (the same kernels; its
C ABI adds include/fbm_secagg_test.h: host runs of device routines, the calling thread's engine
switches, the per-kernel event timer) is `load_test()`; inside `with test_hooks():` the calling
thread's `load()` returns it too, so a whole computation (the bench's timed-kernel step, a test
pinned to one engine) runs through one library.  FBM_TEST_HOOKS=1 routes every thread there.

torch is imported first so that the process has exactly one HIP runtime: torch's
bundled `libamdhip64.so` has the same SONAME (`libamdhip64.so.7`) our library links
against, so the dynamic loader binds us to the already-loaded copy.
"""

import ctypes
import os
import threading

import torch  # noqa: F401  (loads the HIP runtime the library must share)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libfbm_secagg.so")
TEST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libfbm_secagg_test.so")


def ab_variant() -> bool:
    """An A/B measurement of a kernel variant (tools/ab.sh) sets FBM_AB_VARIANT=1 next to
    FBM_LIB_PATH: only then may the library lack newer symbols or be one ABI older."""
    return os.environ.get("FBM_AB_VARIANT") == "1"


def lib_path() -> str:
    """FBM_LIB_PATH (another build of this library) or the in-tree one."""
    return os.environ.get("FBM_LIB_PATH") or LIB_PATH


def test_lib_path() -> str:
    """FBM_LIB_PATH (an A/B variant: built with the test build's exports, tools/ab.sh) or the in-tree
    test build."""
    return os.environ.get("FBM_LIB_PATH") or TEST_LIB_PATH


ABI_VERSION = 7  # include/fbm_secagg.h FBM_ABI_VERSION
TAU_LIMBS = 256  # FBM_TAU_LIMBS: the JL round's 32-bit words (< 2^8192)
FBM_OK = 0
FBM_E_ARG = -1
FBM_E_HIP = -2
FBM_E_RANGE = -3
FBM_E_OVERFLOW = -4
FBM_E_FDH = -5
FBM_E_INVERSE = -6
FBM_E_ITER = -7
FBM_E_UNSUPPORTED = -8
FBM_E_ROUND = -9

FBM_F32 = 0
FBM_F64 = 1
FBM_U64 = 2
FBM_I64 = 3
FBM_U128 = 4
FBM_PT = 5
STATS_WORDS = 4

_lock = threading.Lock()
_libs = {}  # path -> CDLL
_typed = {}  # path -> names whose restype / argtypes are set
_tls = threading.local()  # .test: depth of test_hooks() on this thread
loaded_abi = None  # fbm_abi_version() of the loaded library (ABI_VERSION, or one less for an A/B variant)

c_u64 = ctypes.c_uint64
c_dbl = ctypes.c_double
c_int = ctypes.c_int
c_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/fbm_secagg.h exactly
SIGNATURES = {
    "fbm_abi_version": (c_int, []),
    "fbm_jl_clear_caches": (None, []),
    "fbm_jl_batch_begin": (c_int, []),
    "fbm_jl_batch_abort": (None, []),
    "fbm_jl_batch_count": (c_int, []),
    "fbm_jl_batch_workspace": (c_u64, []),
    "fbm_jl_batch_flush": (c_int, [c_vp, c_u64, c_vp]),
    "fbm_last_error": (ctypes.c_char_p, []),
    "fbm_check_stats": (c_int, [c_vp, c_int, c_vp]),
    "fbm_lom_protect": (c_int, [c_vp, c_int, c_u64, c_dbl, c_dbl, c_dbl, c_u64, c_u64, c_vp, c_vp, c_int, c_int,
                                c_vp, c_u64, c_u64, c_vp, c_vp, c_vp]),
    "fbm_prf_key": (c_int, [c_vp, c_vp, c_u64, c_vp, c_vp]),
    "fbm_dequantize": (c_int, [c_vp, c_u64, c_dbl, c_dbl, c_vp, c_vp]),
    "fbm_lom_aggregate": (c_int, [c_vp, c_int, c_u64, c_u64, c_dbl, c_dbl, c_vp, c_vp, c_vp, c_vp]),
    # host-buffer LOM calls, synchronous (ABI 6)
    "fbm_lom_host_workspace": (c_u64, [c_u64, c_int]),
    "fbm_lom_protect_host": (c_int, [c_vp, c_int, c_u64, c_dbl, c_dbl, c_dbl, c_u64, c_u64, c_vp, c_vp, c_int,
                                     c_int, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp, c_vp]),
    "fbm_lom_aggregate_host": (c_int, [c_vp, c_int, c_u64, c_u64, c_dbl, c_dbl, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_encrypt_workspace": (c_u64, [c_u64]),
    "fbm_jl_aggregate_workspace": (c_u64, [c_u64]),
    # the JL round (tau) is a HOST pointer to TAU_LIMBS limbs (< 2^8192, ABI 3)
    "fbm_jl_encrypt": (c_int, [c_vp, c_int, c_u64, c_dbl, c_dbl, c_dbl, c_u64, c_u64, c_int, c_int, c_vp, c_vp,
                               c_int, c_vp, c_u64, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_encrypt_phase": (c_int, [c_vp, c_int, c_u64, c_dbl, c_dbl, c_dbl, c_u64, c_u64, c_int, c_int, c_vp,
                                     c_vp, c_int, c_vp, c_u64, c_vp, c_vp, c_vp, c_vp, c_int]),
    "fbm_jl_encrypt_factor": (c_int, [c_vp, c_int, c_u64, c_dbl, c_dbl, c_dbl, c_u64, c_u64, c_int, c_int, c_vp,
                                      c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_aggregate": (c_int, [c_vp, c_int, c_u64, c_int, c_int, c_u64, c_vp, c_vp, c_int, c_vp, c_u64, c_u64,
                                 c_dbl, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_decrypt_factor": (c_int, [c_u64, c_vp, c_vp, c_int, c_vp, c_u64, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_decrypt_factor_phase": (c_int, [c_u64, c_vp, c_vp, c_int, c_vp, c_u64, c_vp, c_vp, c_vp, c_vp, c_int]),
    "fbm_jl_aggregate_factor": (c_int, [c_vp, c_int, c_u64, c_int, c_int, c_u64, c_vp, c_vp, c_u64, c_dbl, c_dbl,
                                        c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_pack": (c_int, [c_vp, c_int, c_u64, c_int, c_int, c_vp, c_vp, c_vp]),
    "fbm_jl_unpack": (c_int, [c_vp, c_u64, c_int, c_int, c_u64, c_vp, c_vp]),
    "fbm_jl_fdh": (c_int, [c_u64, c_vp, c_int, c_vp, c_u64, c_vp, c_vp, c_vp]),
    "fbm_jl_fdh_msg": (c_int, [c_u64, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp]),
    "fbm_jl_fdh_msg_row_words": (c_int, [c_int]),
    "fbm_int_true_div_big": (c_int, [c_vp, c_u64, c_vp, c_int, c_int, c_vp, c_vp]),
    "fbm_ves_pack": (c_int, [c_vp, c_u64, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp]),
    "fbm_ves_unpack": (c_int, [c_vp, c_u64, c_int, c_int, c_int, c_u64, c_int, c_vp, c_vp]),
    "fbm_jl_product": (c_int, [c_vp, c_int, c_u64, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_decrypt": (c_int, [c_vp, c_int, c_u64, c_vp, c_vp, c_int, c_vp, c_u64, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_powmod": (c_int, [c_vp, c_vp, c_u64, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    "fbm_jl_decrypt_with": (c_int, [c_vp, c_int, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_int_ops": (c_int, [c_vp, c_u64, c_u64, c_int, c_vp, c_vp, c_vp]),
    "fbm_ass_split": (c_int, [c_vp, c_int, c_u64, c_int, c_int, c_vp, c_vp, c_u64, c_vp, c_vp]),
    "fbm_ass_reconstruct": (c_int, [c_vp, c_int, c_u64, c_vp, c_vp]),
    "fbm_ass_split_wide": (c_int, [c_vp, c_u64, c_int, c_int, c_int, c_int, c_vp, c_vp, c_u64, c_vp, c_vp]),
    "fbm_ass_reconstruct_wide": (c_int, [c_vp, c_int, c_int, c_u64, c_vp, c_vp]),
}

# include/fbm_secagg_test.h: exported by the test build only
TEST_SIGNATURES = {
    "fbm_jl_window": (c_int, []),
    "fbm_jl_mads": (c_int, [c_int]),
    "fbm_jl_quad_mads": (c_int, [c_int]),
    "fbm_jl_triple_mads": (c_int, [c_int]),
    "fbm_jl_set_engine": (c_int, [c_int]),
    "fbm_jl_set_short": (c_int, [c_int]),
    "fbm_jl_engine_for": (c_int, [c_u64]),
    "fbm_test_true_div_big": (c_int, [c_vp, c_u64, c_vp, c_int, c_int, c_vp]),
    "fbm_test_modinv": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "fbm_test_nadic_consts": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_test_short_consts": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_test_short_cache": (c_int, [c_vp, c_int]),
    "fbm_test_fdh_gcd": (c_int, [c_vp, c_vp, c_vp]),
    "fbm_test_gen_exp": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp]),
    "fbm_test_gen_combine": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp]),
    "fbm_test_lom_aggregate_kernel": (c_int, [c_int, c_u64, c_vp, ctypes.c_char_p, c_int]),
    "fbm_prof_enable": (c_int, [c_int]),
    "fbm_prof_report": (c_int, [ctypes.c_char_p, c_int]),
}


class NativeUnavailable(RuntimeError):
    """The HIP extension is not built or cannot be loaded."""


def _open(path: str, sigs: dict) -> ctypes.CDLL:
    """Loads (once per path) a build of the library; it must export every symbol of `sigs` and report
    ABI_VERSION, unless FBM_AB_VARIANT=1."""
    global loaded_abi
    lib = _libs.get(path)
    if lib is not None and _typed[path] >= sigs.keys():  # loaded, every signature of `sigs` set
        return lib
    with _lock:
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"HIP extension not built: {path} is missing (run `python -m fedbiomed_amd._build`)")
        try:
            lib = _libs.get(path) or ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeUnavailable(f"cannot load {path}: {e}") from e
        variant = ab_variant()  # an A/B build (tools/ab.sh) may predate newer symbols
        missing = []
        for name, (res, args) in sigs.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                missing.append(name)
                continue
            fn.restype = res
            fn.argtypes = args
        if missing and not variant:
            raise NativeUnavailable(f"{path} lacks {len(missing)} entry point(s) of its header(s): "
                                    f"{', '.join(missing[:4])}{' ...' if len(missing) > 4 else ''}")
        if "fbm_abi_version" in missing:
            raise NativeUnavailable(f"{path} does not export fbm_abi_version")
        abi = lib.fbm_abi_version()
        # (an A/B variant may be one ABI older: ABI 2 reads the first 16 of the round's limbs, so the
        #  device layer refuses rounds >= 2^512 with it -- _device._check_round)
        if abi != ABI_VERSION and not (variant and abi == ABI_VERSION - 1):
            raise NativeUnavailable(f"ABI version mismatch: {path} reports {abi}, this binding needs {ABI_VERSION}")
        loaded_abi = abi
        _typed[path] = _typed.get(path, set()) | (set(sigs) - set(missing))
        if variant:
            _typed[path] |= set(sigs)  # (an A/B variant may lack some: don't look again)
        _libs[path] = lib
        return lib


def load(path: str = None) -> ctypes.CDLL:
    """The product library (include/fbm_secagg.h), loaded once; raises NativeUnavailable.  Inside
    test_hooks() on this thread, or with FBM_TEST_HOOKS=1, the test build instead (load_test())."""
    if path is None and (getattr(_tls, "test", 0) or os.environ.get("FBM_TEST_HOOKS") == "1"):
        return load_test()
    return _open(path or lib_path(), SIGNATURES)


def load_test() -> ctypes.CDLL:
    """The test build (include/fbm_secagg.h + include/fbm_secagg_test.h): the test suite's host
    hooks, the calling thread's engine / short-path switches, the per-kernel event timer."""
    return _open(test_lib_path(), {**SIGNATURES, **TEST_SIGNATURES})


class test_hooks:
    """Routes this thread's load() to the test build for the duration (re-entrant), so every
    library call of a computation goes through the library whose switches / timer it sets:

        with _native.test_hooks():
            _native.prof_enable(True)
            ...
    """

    def __enter__(self):
        load_test()
        _tls.test = getattr(_tls, "test", 0) + 1
        return self

    def __exit__(self, *exc):
        _tls.test -= 1
        return False


def last_error() -> str:
    return (load().fbm_last_error() or b"").decode(errors="replace")


def prof_enable(on: bool) -> None:
    """The test build's per-kernel event timer (calls made through load_test() / test_hooks())."""
    load_test().fbm_prof_enable(1 if on else 0)


def prof_report() -> dict:
    """{kernel: (launches, total_ms)} of the test build's launches recorded since the last report."""
    lib = load_test()
    need = lib.fbm_prof_report(None, 0)  # non-destructive size query
    buf = ctypes.create_string_buffer(need + 4096)
    lib.fbm_prof_report(buf, len(buf))
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split()
        out[name] = (int(cnt), float(ms))
    return out
