"""ctypes binding of the C-ABI HIP library (include/fbm_secagg.h).

The library is built in-tree (`python -m fedbiomed_amd._build` or
`__graft_entry__.build()`) to `fedbiomed_amd/_lib/libfbm_secagg.so`.  There is NO
CPU fallback: if the library or a GPU is missing, every compute call raises.

torch is imported first so that the process has exactly one HIP runtime: torch's
bundled `libamdhip64.so` has the same SONAME (`libamdhip64.so.7`) our library links
against, so the dynamic loader binds us to the already-loaded copy.
"""

import ctypes
import os
import threading

import torch  # noqa: F401  (loads the HIP runtime the library must share)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libfbm_secagg.so")


def ab_variant() -> bool:
    """An A/B measurement of a kernel variant (tools/ab.sh) sets FBM_AB_VARIANT=1 next to
    FBM_LIB_PATH: only then may the library lack newer symbols or be one ABI older."""
    return os.environ.get("FBM_AB_VARIANT") == "1"


def lib_path() -> str:
    """FBM_LIB_PATH (another build of this library) or the in-tree one."""
    return os.environ.get("FBM_LIB_PATH") or LIB_PATH


ABI_VERSION = 6  # include/fbm_secagg.h FBM_ABI_VERSION
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
_lib = None
loaded_abi = None  # fbm_abi_version() of the loaded library (ABI_VERSION, or one less for an A/B variant)

c_u64 = ctypes.c_uint64
c_dbl = ctypes.c_double
c_int = ctypes.c_int
c_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/fbm_secagg.h exactly
SIGNATURES = {
    "fbm_abi_version": (c_int, []),
    "fbm_jl_window": (c_int, []),
    "fbm_jl_mads": (c_int, [c_int]),
    "fbm_jl_quad_mads": (c_int, [c_int]),
    "fbm_jl_triple_mads": (c_int, [c_int]),
    "fbm_jl_set_engine": (c_int, [c_int]),
    "fbm_jl_set_short": (c_int, [c_int]),
    "fbm_jl_clear_caches": (None, []),
    "fbm_jl_engine_for": (c_int, [c_u64]),
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
    "fbm_test_true_div_big": (c_int, [c_vp, c_u64, c_vp, c_int, c_int, c_vp]),
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
    "fbm_test_modinv": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "fbm_test_nadic_consts": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_test_short_consts": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "fbm_test_short_cache": (c_int, [c_vp, c_int]),
    "fbm_test_fdh_gcd": (c_int, [c_vp, c_vp, c_vp]),
    "fbm_test_gen_exp": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp]),
    "fbm_test_gen_combine": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp]),
    "fbm_prof_enable": (c_int, [c_int]),
    "fbm_prof_report": (c_int, [ctypes.c_char_p, c_int]),
}


class NativeUnavailable(RuntimeError):
    """The HIP extension is not built or cannot be loaded."""


def load(path: str = None) -> ctypes.CDLL:
    """Loads (once) and returns the C-ABI library; raises NativeUnavailable.  The library must
    export every symbol of SIGNATURES and report ABI_VERSION, unless FBM_AB_VARIANT=1."""
    global _lib, loaded_abi
    with _lock:
        if _lib is not None:
            return _lib
        path = path or lib_path()
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"HIP extension not built: {path} is missing (run `python -m fedbiomed_amd._build`)")
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeUnavailable(f"cannot load {path}: {e}") from e
        variant = ab_variant()  # an A/B build (tools/ab.sh) may predate newer symbols
        missing = []
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                missing.append(name)
                continue
            fn.restype = res
            fn.argtypes = args
        if missing and not variant:
            raise NativeUnavailable(f"{path} lacks {len(missing)} entry point(s) of include/fbm_secagg.h: "
                                    f"{', '.join(missing[:4])}{' ...' if len(missing) > 4 else ''}")
        if "fbm_abi_version" in missing:
            raise NativeUnavailable(f"{path} does not export fbm_abi_version")
        abi = lib.fbm_abi_version()
        # (an A/B variant may be one ABI older: ABI 2 reads the first 16 of the round's limbs, so the
        #  device layer refuses rounds >= 2^512 with it -- _device._check_round)
        if abi != ABI_VERSION and not (variant and abi == ABI_VERSION - 1):
            raise NativeUnavailable(f"ABI version mismatch: {path} reports {abi}, this binding needs {ABI_VERSION}")
        loaded_abi = abi
        _lib = lib
        return lib


def last_error() -> str:
    return (load().fbm_last_error() or b"").decode(errors="replace")


def prof_enable(on: bool) -> None:
    load().fbm_prof_enable(1 if on else 0)


def prof_report() -> dict:
    """{kernel: (launches, total_ms)} of the launches recorded since the last report."""
    lib = load()
    need = lib.fbm_prof_report(None, 0)  # non-destructive size query
    buf = ctypes.create_string_buffer(need + 4096)
    lib.fbm_prof_report(buf, len(buf))
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split()
        out[name] = (int(cnt), float(ms))
    return out
