"""Device-resident entry points: torch tensors in HBM -> C-ABI HIP kernels -> torch tensors.

torch is plumbing here (device memory, the current HIP stream); all arithmetic runs in the
hand-written gfx950 kernels of `fedbiomed_amd/csrc` behind `include/fbm_secagg.h`.  There is
no CPU fallback: without a visible HIP device every call raises `NativeUnavailable`.

Host-side work in this module is limited to argument validation and the per-call uniform
parameters the reference computes in Python (`float(c)`, `(2c)/(T-1)`, slot sizes), so the
Python semantics stay bit-identical.
"""

from __future__ import annotations

import array
import ctypes
import logging
import math
import operator
import os
import sys
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from .constants import ErrorNumbers, SAParameters
from .exceptions import FedbiomedSecaggCrypterError, FedbiomedSecaggError

U64_MAX = 2**64 - 1
FBM_WARN_CLIPPED = 16  # stats flag: some |x| > clipping range (a warning, not an error)
FBM_STAT_MAXBITS, FBM_STAT_ERRFLAGS = 0, 1  # status words (csrc/fbm_internal.hpp)

logger = logging.getLogger("fedbiomed_amd")


# ------------------------------------------------------------------------------------------
# plumbing
# ------------------------------------------------------------------------------------------
def device() -> torch.device:
    if not torch.cuda.is_available():
        raise N.NativeUnavailable("no HIP device is visible: the MI355X crypter has no CPU path")
    N.load()
    return torch.device("cuda", torch.cuda.current_device())


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t: Optional[torch.Tensor]) -> Optional[ctypes.c_void_p]:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _np_ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _raise(rc: int) -> None:
    msg = N.last_error()
    if rc == N.FBM_E_OVERFLOW:
        raise FedbiomedSecaggError(f"{ErrorNumbers.FB417.value}: {msg}")
    if rc == N.FBM_E_RANGE:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: Cannot reverse quantize, received values exceed maximum number")
    if rc == N.FBM_E_FDH:
        raise OverflowError("int too big to convert")  # the reference's FDH counter.to_bytes(1)
    if rc == N.FBM_E_INVERSE:
        raise ZeroDivisionError("invert() no inverse exists")
    if rc == N.FBM_E_ROUND:
        raise OverflowError("int too big to convert")  # the reference's (i + tau).to_bytes(8, 'big')
    if rc in (N.FBM_E_ARG, N.FBM_E_UNSUPPORTED):
        raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: {msg}")
    raise RuntimeError(f"fedbiomed_amd HIP error {rc}: {msg}")


def _call(fn, *args) -> None:
    rc = fn(*args)
    if rc != N.FBM_OK:
        _raise(rc)


class deferred_checks:
    """Within this context the device status words of JL / LOM encrypts are checked once, at exit,
    instead of after every call (each check synchronises its stream).  This lets the
    encrypts of several parties issued on different HIP streams overlap on the GPU; any
    error is still raised, from the `with` statement's exit.

        with D.deferred_checks():
            for p, s in enumerate(streams):
                with torch.cuda.stream(s):
                    cts[p] = D.jl_encrypt(...)
    """

    _tls = threading.local()  # per thread: another thread's calls keep their own checks

    def __init__(self, merge: bool = False):
        """merge: the calls inside are stripes of ONE logical call (the list API's overlapped encrypt):
        their status words are combined -- error flags OR-ed, the max bit length maxed -- and checked
        once, so a clipping warning is logged once per call, as the reference logs it."""
        self._merge = merge

    @staticmethod
    def _stack() -> List[list]:
        st = getattr(deferred_checks._tls, "stack", None)
        if st is None:
            st = deferred_checks._tls.stack = []
        return st

    def __enter__(self):
        deferred_checks._stack().append([])
        return self

    def __exit__(self, exc_type, exc, tb):
        pending = deferred_checks._stack().pop()
        if not pending:
            return False
        # wait for the streams that wrote the status words only (an event recorded after
        # each), not the whole device: other threads' work keeps running
        for _, _, ev in pending:
            ev.synchronize()
        # the status words were copied to pinned host memory behind their kernels (_check_stats_or_defer):
        # no device work and no copy here; a device tensor (adopted from elsewhere) is copied now
        host = np.stack([(st if st.device.type == "cpu" else st.cpu()).numpy() for st, _, _ in pending])
        if self._merge:
            assert len({nodes for _, (nodes, _), _ in pending}) == 1 and all(p is None for _, (_, p), _ in pending)
            row = host[:1].copy()
            row[0, FBM_STAT_MAXBITS] = host[:, FBM_STAT_MAXBITS].astype(np.uint32).max()
            row[0, FBM_STAT_ERRFLAGS] = np.bitwise_or.reduce(host[:, FBM_STAT_ERRFLAGS].astype(np.uint32))
            pending, host = pending[:1], row
        try:
            for (_, (nodes, post), _), row in zip(pending, host):
                _check_stats_host(row, nodes)
                if post is not None:
                    raise post
        except Exception as dev_err:
            if exc is not None:  # the device condition came first: surface it, chained
                raise dev_err from exc
            raise
        return False


class capture_checks(deferred_checks):
    """deferred_checks whose status words are NOT checked at exit but kept in `.pending`, for work
    issued ahead of the call that uses it (SecaggCrypter.prepare_aggregate): that call hands them to
    adopt_checks() inside its own deferred_checks, so a device condition of the early work is raised
    by the call that consumes it, in its place."""

    def __exit__(self, exc_type, exc, tb):
        self.pending = deferred_checks._stack().pop()
        return False


def adopt_checks(pending: list) -> None:
    """Status words captured by capture_checks: into the current deferred_checks context, or checked
    now (waiting for their streams) when there is none."""
    active = deferred_checks._stack()
    if active:
        active[-1].extend(pending)
        return
    for st, (nodes, post), ev in pending:
        ev.synchronize()
        _check_stats_host(st.cpu().numpy(), nodes)
        if post is not None:
            raise post


def _check_stats_or_defer(stats: torch.Tensor, lom_nodes: int = 0, post: Optional[Exception] = None) -> None:
    """`post`: a host-known error of the same call, raised after the device conditions (the
    reference's order, e.g. LOM's round-counter overflow after its overflow guard)."""
    active = deferred_checks._stack()
    if active:
        if stats.device.type != "cpu":  # to pinned host memory on the current stream, right behind the
            host = host_empty(stats.shape, stats.dtype)  # kernels that write it: the exit reads it without
            host.copy_(stats, non_blocking=True)  # a copy of its own (one synchronisation less per call)
            stats = host
        ev = torch.cuda.Event()
        ev.record()  # on the current stream, after the kernels (and the copy)
        active[-1].append((stats, (lom_nodes, post), ev))
    else:
        _check_stats(stats, lom_nodes)
        if post is not None:
            raise post


def _check_stats(stats: torch.Tensor, lom_nodes: int = 0) -> int:
    return _check_stats_host(stats.cpu().numpy(), lom_nodes)  # .cpu() synchronises the stream


def _check_stats_host(host: np.ndarray, lom_nodes: int = 0) -> int:
    host = np.ascontiguousarray(host).astype(np.uint32)
    if int(host[1]) & FBM_WARN_CLIPPED:  # _check_clipping_range (utils/_secagg_utils.py:189-204)
        logger.warning("There are some numbers in the local vector that exceeds clipping range. "
                       "Please increase the clipping range to account for value")
    mb = ctypes.c_uint32(0)
    rc = N.load().fbm_check_stats(_np_ptr(host), lom_nodes, ctypes.byref(mb))
    if rc == N.FBM_E_OVERFLOW:
        raise FedbiomedSecaggError(_lom_overflow_message(int(mb.value), lom_nodes))
    if rc != N.FBM_OK:
        _raise(rc)
    return int(mb.value)


def _lom_overflow_message(max_bits: int, num_nodes: int) -> str:
    """LOM.protect's overflow-guard message (secagg/_lom.py:133-149), word for word."""
    node_bits = math.ceil(math.log2(num_nodes))
    avail = 64 - node_bits
    missing = max_bits + node_bits - 64
    return (f"{ErrorNumbers.FB417.value}: Secure aggregation overflow detected.\n\n"
            f"Your value requires {max_bits} bits, but only {avail} bits "
            f"are available (64-bit dtype minus {node_bits} bits reserved for {num_nodes} nodes).\n\n"
            f"To fix this, choose one of the following:\n"
            f"  1) Reduce the number of nodes to at most {2 ** (64 - max_bits)} (currently {num_nodes}).\n"
            f"  2) Reduce your values by at least {missing} bit(s) "
            f"(i.e. divide them by at least {2 ** missing}).\n"
            f"  3) If you are quantizing model weights, use a lower quantization range "
            f"so that individual values fit within {avail} bits.")


def _stats(dev) -> torch.Tensor:
    return torch.empty(N.STATS_WORDS, dtype=torch.int32, device=dev)


def _x_dtype(x: torch.Tensor) -> int:
    if x.dtype == torch.float32:
        return N.FBM_F32
    if x.dtype == torch.float64:
        return N.FBM_F64
    if x.dtype in (torch.int64, torch.uint64):
        return N.FBM_U64
    raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: unsupported input dtype {x.dtype}")


# ------------------------------------------------------------------------------------------
# parameters (Python-exact, as the reference computes them)
# ------------------------------------------------------------------------------------------
def quant_params(clip, target) -> Tuple[float, float, float, int]:
    """(float(c), float(2c), float(T), T-1) for `quantize` (utils/_secagg_utils.py:82-119)."""
    c = SAParameters.CLIPPING_RANGE if clip is None else clip
    if target - 1 > U64_MAX:
        # the reference's np.vectorize(otypes=[uint64]) raises on the clipped elements
        raise OverflowError("Python int too large to convert to C unsigned long")
    if c == 0:
        raise ZeroDivisionError("float division by zero")
    cf = float(c)
    if cf != c or abs(cf) > 2.0**53 or c < 0:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: clipping_range must be a positive value exactly representable "
            f"in float64 for the device quantiser (got {c!r})")
    return cf, float(2 * c), float(target), int(target - 1)


def dequant_params(clip, target) -> Tuple[float, float]:
    """(float(-c), (2c)/(T-1)) for `reverse_quantize` (utils/_secagg_utils.py:168-182)."""
    c = SAParameters.CLIPPING_RANGE if clip is None else clip
    step = (c - (-c)) / (target - 1)  # Python int/int true division, correctly rounded
    return float(-c), float(step)


def jl_slot(target: Optional[int], n_users: int) -> Tuple[int, int]:
    """(element_size, comp_ratio) of the JL vector encoder (_jls.py:104-116, 587-591)."""
    target = target or SAParameters.TARGET_RANGE
    valuesize = math.ceil(math.log2(target) + math.log2(SAParameters.WEIGHT_RANGE))
    es = valuesize + math.ceil(math.log2(n_users + 1))
    cr = math.floor((SAParameters.KEY_SIZE // 2) / es)
    return es, cr


def int_limbs(v: int, n_limbs: int) -> np.ndarray:
    return np.frombuffer(int(v).to_bytes(4 * n_limbs, "little"), dtype=np.uint32).copy()


# ------------------------------------------------------------------------------------------
# list <-> tensor conversions (the host-memory boundary, measured in DESIGN.md)
# ------------------------------------------------------------------------------------------
class _PyConvFallback:
    """Pure-Python versions of csrc/fbm_pyconv.c's three loops (same contracts), used when
    the C module is not built for this interpreter.  Host list <-> buffer conversions only:
    no secagg arithmetic happens here."""

    @staticmethod
    def all_ints(seq: list) -> bool:
        return all(isinstance(v, int) for v in seq)

    @staticmethod
    def all_ints_lists(lists: list) -> int:
        if not all(isinstance(r, list) for r in lists):
            raise TypeError("all_ints_lists takes a list of lists")
        return next((u for u, r in enumerate(lists) if not all(isinstance(v, int) for v in r)), -1)

    @staticmethod
    def floats_to_f64(seq: list, out: np.ndarray) -> int:
        if out.nbytes != 8 * len(seq):
            raise ValueError(f"output buffer holds {out.nbytes} bytes, {8 * len(seq)} needed")
        for i, v in enumerate(seq):
            if not isinstance(v, float):
                return i
        out[:] = np.asarray(seq, dtype=np.float64) if seq else out[:0]
        return -1

    @staticmethod
    def ints_to_bytes(seq: list, nb: int, out: np.ndarray) -> int:
        if nb <= 0:
            raise ValueError("width must be positive")
        if out.nbytes != nb * len(seq):
            raise ValueError(f"output buffer holds {out.nbytes} bytes, {nb * len(seq)} needed")
        dst = out.reshape(-1).view(np.uint8)
        for i, v in enumerate(seq):
            if not isinstance(v, int) or v < 0 or v.bit_length() > 8 * nb:
                return i
            dst[i * nb:(i + 1) * nb] = np.frombuffer(v.to_bytes(nb, "little"), dtype=np.uint8)
        return -1

    @staticmethod
    def bytes_to_ints(buf, nb: int) -> list:
        b = memoryview(buf).cast("B").tobytes()
        if nb <= 0 or len(b) % nb:
            raise ValueError("buffer is not a whole number of values")
        return [int.from_bytes(b[i:i + nb], "little") for i in range(0, len(b), nb)]

    @staticmethod
    def ints_to_bytes_held(lists: list, lo: int, hi: int, nb: int, out: np.ndarray) -> int:
        if nb <= 0 or nb % 4 or lo < 0 or hi < lo:
            raise ValueError("bad range or width (a positive multiple of 4 bytes)")
        if not all(isinstance(v, list) and len(v) >= hi for v in lists):
            raise ValueError("every item must be a list holding the range")
        m = hi - lo
        if out.nbytes != len(lists) * m * nb:
            raise ValueError(f"output buffer holds {out.nbytes} bytes, {len(lists) * m * nb} needed")
        rows = out.reshape(len(lists), m * nb // out.itemsize) if lists else out
        for u, v in enumerate(lists):
            b = _PyConvFallback.ints_to_bytes(v[lo:hi], nb, rows[u])
            if b >= 0:
                return u * m + b
        return -1

    @staticmethod
    def float_pool(n: int) -> list:
        if n < 0:
            raise ValueError("negative length")
        return [float(0) for _ in range(n)]

    @staticmethod
    def none_list(n: int) -> list:
        if n < 0:
            raise ValueError("negative length")
        return [None] * n

    @staticmethod
    def f64_into_list(lst: list, off: int, buf) -> None:
        a = np.frombuffer(memoryview(buf).cast("B"), dtype=np.float64)
        if off < 0 or off + len(a) > len(lst):
            raise ValueError("float64 buffer does not fit the list at that offset")
        if any(v is not None and type(v) is not float for v in lst[off:off + len(a)]):
            raise ValueError("f64_into_list fills slots that hold None or floats only")
        lst[off:off + len(a)] = a.tolist()


def _pyconv():
    """The list API's C conversion loops (csrc/fbm_pyconv.c), built in-tree by _build; the
    pure-Python equivalents when the module is absent (not built for this interpreter)."""
    global _PYCONV
    if _PYCONV is None:
        import importlib.util

        from ._build import PYCONV_OUT

        if not os.path.exists(PYCONV_OUT) or os.environ.get("FBM_NO_PYCONV"):
            logger.info("fedbiomed_amd: %s not built; list conversions run in Python", PYCONV_OUT)
            _PYCONV = _PyConvFallback
            return _PYCONV
        spec = importlib.util.spec_from_file_location("_fbm_pyconv", PYCONV_OUT)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.set_conv_threads(min(16, host_cpu_share()))
        _PYCONV = mod
    return _PYCONV


def cgroup_cpu_quota() -> Optional[float]:
    """CPUs' worth of CPU time the process's cgroup allows (cgroup v2 cpu.max, v1 cfs quota / period),
    or None when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            per = int(fh.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def host_cpu_share() -> int:
    """The CPUs this process may use: its affinity, capped by its cgroup's CPU quota (>= 1).  The list
    API's host conversions use up to 16 of them (the 10M x 8 list aggregate with its factor prepared:
    43.8 ms on 8 threads, 37.8 ms on 16 -- profiles/archive/r5aj_list_agg_prepared.jsonl)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    return max(1, min(avail, int(quota)) if quota else avail)


_PYCONV = None


def host_empty(shape, dtype: torch.dtype) -> torch.Tensor:
    """Host staging buffer for the list API: pinned (torch's caching host allocator hands the
    same pages back call after call -- no first-touch page faults, DMA-direct copies) when a
    HIP device is visible, plain memory otherwise (the argument checks run without one)."""
    return torch.empty(shape, dtype=dtype, pin_memory=torch.cuda.is_available())


def to_host(t: torch.Tensor) -> torch.Tensor:
    """Device tensor -> host copy through a (cached) pinned staging buffer."""
    host = host_empty(t.shape, t.dtype)
    host.copy_(t)
    return host


def all_ints(seq: list) -> bool:
    """all(isinstance(v, int) for v in seq) of a list, in one C pass (csrc/fbm_pyconv.c)."""
    return bool(_pyconv().all_ints(seq))


def all_ints_lists(lists: list) -> bool:
    """Every item of every list (a list of lists) is an int (isinstance), in one C pass over host threads."""
    return _pyconv().all_ints_lists(lists) < 0


def floats_to_host(params: list) -> Optional[torch.Tensor]:
    """List of floats -> float64 host tensor in one C pass; None if an item is not a float
    (isinstance(v, float), subclasses included -- the reference's check)."""
    host = host_empty(len(params), torch.float64)
    return host if _pyconv().floats_to_f64(params, host.numpy()) < 0 else None


def floats_to_device(params: Sequence[float], dev=None) -> torch.Tensor:
    """Validated list of floats -> float64 device tensor."""
    dev = dev or device()
    host = floats_to_host(params) if isinstance(params, list) else None
    if host is None:  # not a list, or not all floats: numpy's conversion (raises the TypeError)
        host = torch.from_numpy(np.frombuffer(array.array("d", params), dtype=np.float64))
    return host.to(dev)


def u64_to_host(rows) -> Tuple[torch.Tensor, bool]:
    """list[int] or list[list[int]] -> host int64 tensor holding the uint64 bit patterns, and whether it
    is the pinned staging block.  np.array(..., dtype=uint64) raises exactly where the reference's
    conversion raises."""
    if isinstance(rows, list) and rows and all(isinstance(r, list) for r in rows) and \
            len(set(map(len, rows))) == 1:  # fast path: equal-length rows of in-range ints
        host = host_empty((len(rows), len(rows[0])), torch.int64)
        buf = host.numpy()
        if all(_pyconv().ints_to_bytes(r, 8, buf[u]) < 0 for u, r in enumerate(rows)):
            return host, True
    arr = np.array(rows, dtype=np.uint64)  # anything else, with numpy's exact errors
    return torch.from_numpy(arr.view(np.int64)), False


def u64_to_device(rows, dev=None) -> torch.Tensor:
    """u64_to_host's tensor on the device."""
    dev = dev or device()
    host, pinned = u64_to_host(rows)
    return host.to(dev, non_blocking=pinned)  # stream-ordered (the pinned block is held until it lands)


def u64_from_device(t: torch.Tensor) -> List[int]:
    return to_host(t).numpy().view(np.uint64).tolist()


def ints_to_limbs(cts: Sequence[int], modulus: Optional[int] = None, out: Optional[np.ndarray] = None) -> np.ndarray:
    """JL ciphertext ints -> [n, 64] uint32 little-endian limbs (into `out` if given, e.g. a
    party's row of the aggregate's input).  Values outside [0, 2^2048) are reduced mod N^2
    first (same residue, as the reference reduces in its product); in-range values go
    through unchanged."""
    if out is None:
        out = np.empty((len(cts), 64), dtype=np.uint32)
    cts = cts if isinstance(cts, list) else list(cts)
    bad = _pyconv().ints_to_bytes(cts, 256, out)  # common case: one C pass, -1
    while bad >= 0:  # an out-of-range (or non-int) value: reduce it, continue after it
        c = int(cts[bad])
        if c < 0 or c.bit_length() > 2048:
            if modulus is None:
                raise OverflowError("ciphertext outside [0, 2^2048) and no modulus to reduce it by")
            c %= modulus
        out[bad] = np.frombuffer(c.to_bytes(256, "little"), dtype=np.uint32)
        rest = _pyconv().ints_to_bytes(cts[bad + 1:], 256, out[bad + 1:])
        bad = -1 if rest < 0 else bad + 1 + rest
    return out


def convert_stripe(lists: List[list], c0: int, c1: int, modulus: Optional[int], out: np.ndarray) -> np.ndarray:
    """Items [c0, c1) of every party's ciphertext list -> `out` [P, c1 - c0, 64] uint32 limbs on host threads
    in one C call that holds the GIL, so the readers need no pins (csrc/fbm_pyconv.c ints_to_bytes_held);
    then ints_to_limbs' slow path (reduction mod N^2 of out-of-range values) for any party row that has one."""
    bad = _pyconv().ints_to_bytes_held(lists, c0, c1, 256, out)
    if bad >= 0:  # rare: values outside [0, 2^2048) from this party row on
        m = c1 - c0
        for u in range(bad // max(m, 1), len(lists)):
            ints_to_limbs(lists[u][c0:c1], modulus, out=out[u])
    return out


def none_list(n: int) -> list:
    """[None] * n in one C pass: an output list whose float objects f64_into_list makes."""
    return _pyconv().none_list(n)


def float_pool(n: int) -> list:
    """n fresh 0.0 floats held by the returned list only: an aggregate's output list made ahead
    (prepare_aggregate, or made while the GPU exponentiates); f64_into_list then writes its values in
    place, no allocation."""
    return _pyconv().float_pool(n)


def f64_into_list(lst: list, off: int, values: np.ndarray) -> None:
    """lst[off:off + len(values)] = the float64 values as Python floats, in one pass."""
    _pyconv().f64_into_list(lst, off, np.ascontiguousarray(values, dtype=np.float64))


def inplace_allowed(version=None) -> bool:
    """Writes into output objects made ahead -- an int_pool int's digits, a float_pool float's value,
    written by csrc/fbm_pyconv.c before the list is handed out -- only on CPython 3.10 / 3.11, the
    object layouts the module is written and tested against (the C module compiles them out on any
    other version; this refuses them besides, whatever the build)."""
    import platform

    v = sys.version_info if version is None else version
    return tuple(v[:2]) in ((3, 10), (3, 11)) and platform.python_implementation() == "CPython"


# The unprepared list calls' in-place writes, per call (kept only where they gain >= 10 %).
# Measured at 10M on MI355X (tools/inplace_probe.py, profiles/r6b_inplace_probe.jsonl, interleaved medians of
# 5): the node's JL encrypt 138.4 ms with its int_pool against 143.0 without (3.3 %: off), the researcher's
# aggregate 140.1 ms with its last stripe's floats made while the GPU exponentiates against 157.9 without
# (11.3 %: on).  Off, the call makes every output object with its value; the prepare_* extensions keep
# their pools (their objects are made outside the call).
INPLACE_UNPREPARED = {"encrypt": False, "aggregate": True}


def inplace(prepared: bool, call: str = "encrypt") -> bool:
    """Whether a call may write into output objects made ahead: an interpreter the C module's writes are
    for, a module built with them, and -- for an unprepared call -- INPLACE_UNPREPARED[call]."""
    m = _pyconv()
    if m is _PyConvFallback or not inplace_allowed() or not m.build_flags()[0]:
        return False
    return prepared or bool(INPLACE_UNPREPARED.get(call))


def int_pool(n: int, nbytes: int = 256, prepared: bool = True) -> Optional[list]:
    """n ints with room for nbytes-byte values made ahead (a prepared encrypt's output list: JL
    ciphertexts, 256 bytes, through limbs_into_pool; LOM's masked values, 8 bytes, through
    u64_into_pool), or None where they may not be made (inplace(prepared): the module not built, an
    interpreter other than CPython 3.10 / 3.11, an unprepared encrypt with INPLACE_UNPREPARED off)."""
    return _pyconv().int_pool(n, nbytes) if inplace(prepared) else None


def u64_into_pool(pool: list, arr: np.ndarray) -> list:
    """int_pool(n, 8)'s ints take the uint64 values in place (host threads); the pool -- or a fresh list
    when a pool int is also held elsewhere (it is then never written)."""
    try:
        _pyconv().words_into_pool(pool, np.ascontiguousarray(arr, dtype=np.uint64).view(np.uint32), 8)
    except ValueError:
        return np.asarray(arr, dtype=np.uint64).tolist()
    return pool


def limbs_into_pool(pool: list, arr: np.ndarray, off: int = 0, strict: bool = False) -> list:
    """int_pool's ints [off, off + n) take the [n, 64] uint32 limb rows' values in place (host threads); the
    pool.  When a pool int is also held elsewhere nothing is written and, unless `strict` (a caller that
    fills a private pool by slices: ValueError), a fresh list of the rows' values is returned instead."""
    try:
        _pyconv().words_into_pool(pool, np.ascontiguousarray(arr, dtype=np.uint32), 256, off)
    except ValueError:
        if strict:
            raise
        return limbs_to_ints(arr)
    return pool


def limbs_to_ints(arr: np.ndarray) -> List[int]:
    return _pyconv().bytes_to_ints(np.ascontiguousarray(arr, dtype=np.uint32), 256)


def limbs_to_ints_w(t: torch.Tensor, words: int) -> List[int]:
    """[n, words] 32-bit limbs (device or host tensor) -> list of Python ints."""
    a = (to_host(t) if t.is_cuda else t).numpy().view(np.uint32)
    return _pyconv().bytes_to_ints(np.ascontiguousarray(a.reshape(-1, words)), 4 * words)


# ------------------------------------------------------------------------------------------
# LOM
# ------------------------------------------------------------------------------------------
def _secret_block(secrets: Sequence[bytes]) -> np.ndarray:
    for s in secrets:
        if not isinstance(s, (bytes, bytearray)) or len(s) != 32:
            n = len(s) * 8 if isinstance(s, (bytes, bytearray)) else "?"
            raise FedbiomedSecaggError(
                f"{ErrorNumbers.FB417.value}: Error while ciphering: got exception "
                f"Invalid key size ({n}) for ChaCha20.")
    return np.frombuffer(b"".join(bytes(s) for s in secrets) or b"\0", dtype=np.uint8).copy()


def _nonce_block(nonce: bytes) -> np.ndarray:
    if not isinstance(nonce, (bytes, bytearray)) or len(nonce) != 16:
        raise FedbiomedSecaggError(
            f"{ErrorNumbers.FB417.value}: Error while ciphering: got exception nonce must be 128-bits (16 bytes)")
    return np.frombuffer(bytes(nonce), dtype=np.uint8).copy()


def lom_protect(x: torch.Tensor, secrets: Sequence[bytes], signs: Sequence[int], nonce: bytes, tau: int,
                n_nodes: int, clip=None, target=None, weight: int = 1, raw_seeds: bool = False,
                elem_offset: int = 0, out: Optional[torch.Tensor] = None, check_now: bool = False) -> torch.Tensor:
    """One party's masked vector (u64 bit patterns in an int64 tensor); raises the
    reference's LOM overflow error when max(bit_length(q*w)) >= 64 - ceil(log2(n_nodes)).
    check_now: check the status word before returning even inside `deferred_checks`."""
    dev = x.device
    lib = N.load()
    target = target or SAParameters.TARGET_RANGE
    c, c2, tf, tm1 = quant_params(clip, target) if x.dtype != torch.int64 else (1.0, 2.0, 1.0, 0)
    sec = _secret_block(secrets)
    sg = np.asarray([1 if s > 0 else -1 for s in signs] or [0], dtype=np.int8)
    nb = _nonce_block(nonce)
    x = x.contiguous()
    n = x.numel()
    # PRF.eval_key / eval_vector (_lom.py:43-45, 81) serialise tau and i + tau to 16 / 8 big-endian
    # bytes: a negative tau, or some i + tau >= 2^64, is the reference's OverflowError, raised (like
    # it) after the overflow guard and only when there are peers to mask with.  The C-ABI reports
    # i + tau past 2^64 for a 64-bit tau (FBM_E_ROUND); a tau outside [0, 2^64) is known here.
    post = None
    if secrets and n > 0 and not 0 <= tau <= U64_MAX:
        post = OverflowError("can't convert negative int to unsigned" if tau < 0 else "int too big to convert")
        tau = 0
    tau &= U64_MAX
    if out is not None:  # caller-owned destination, e.g. row p of the aggregate's [P, n] matrix
        if out.dtype != torch.int64 or out.numel() != n or not out.is_contiguous() or out.device != dev:
            raise ValueError("out must be a contiguous int64 tensor of x.numel() elements on x's device")
        y = out
    else:
        y = torch.empty(n, dtype=torch.int64, device=dev)
    st = _stats(dev)
    _call(lib.fbm_lom_protect, _ptr(x), _x_dtype(x), n, c, c2, tf, tm1, int(weight), _np_ptr(sec), _np_ptr(sg),
          len(secrets), 1 if raw_seeds else 0, _np_ptr(nb), int(tau), int(elem_offset), _ptr(y), _ptr(st),
          _stream())
    if check_now:
        _check_stats(st, n_nodes)
        if post is not None:
            raise post
    else:
        _check_stats_or_defer(st, lom_nodes=n_nodes, post=post)
    return y


# Vectors up to this many elements take the one-call host-buffer path of the LOM list API
# (fbm_lom_protect_host / fbm_lom_aggregate_host): a 1 000-element call is launch-bound.
LOM_HOST_CALL_MAX = 1 << 16

_host_ws = {}  # thread ident -> that thread's device workspace of the synchronous host-buffer calls
_host_ws_lock = threading.Lock()


def _host_workspace(nbytes: int, dev) -> torch.Tensor:
    """This thread's device workspace for the synchronous host-buffer calls (one call at a time per
    thread; grown, never shrunk).  It holds a call's plaintext parameters and masked vector only until
    _scrub_host_workspace zeroes it behind the call; release_host_workspaces drops every thread's."""
    key = threading.get_ident()
    with _host_ws_lock:
        ws = _host_ws.get(key)
        if ws is None or ws.numel() < nbytes or ws.device != dev:
            ws = _host_ws[key] = torch.zeros(max(nbytes, 1 << 20), dtype=torch.uint8, device=dev)
    return ws


def _scrub_host_workspace(ws: torch.Tensor, nbytes: int) -> None:
    """Zeroes the bytes a synchronous host-buffer call used (no node's parameters or masked
    vector left in HBM after its call), queued on the call's stream behind it: the call returns without
    waiting for it."""
    ws[:nbytes].zero_()


def release_host_workspaces() -> None:
    """Zeroes and drops every thread's host-call workspace (the clear-caches path)."""
    with _host_ws_lock:
        for ws in _host_ws.values():
            ws.zero_()
        _host_ws.clear()


def lom_protect_host(x: np.ndarray, secrets: Sequence[bytes], signs: Sequence[int], nonce: bytes, tau: int,
                     n_nodes: int, clip=None, target=None, weight: int = 1) -> np.ndarray:
    """lom_protect of a HOST float64 vector into a host uint64 vector, in one synchronous C call
    (copy in, kernel, copy out); the status words checked before returning, as lom_protect(check_now)."""
    dev = device()
    lib = N.load()
    target = target or SAParameters.TARGET_RANGE
    c, c2, tf, tm1 = quant_params(clip, target)
    sec = _secret_block(secrets)
    sg = np.asarray([1 if s > 0 else -1 for s in signs] or [0], dtype=np.int8)
    nb = _nonce_block(nonce)
    x = np.ascontiguousarray(x, dtype=np.float64)
    n = x.shape[0]
    post = None  # (lom_protect's round-counter domain, in the reference's order)
    if secrets and n > 0 and not 0 <= tau <= U64_MAX:
        post = OverflowError("can't convert negative int to unsigned" if tau < 0 else "int too big to convert")
        tau = 0
    tau &= U64_MAX
    blk = host_empty(n + N.STATS_WORDS // 2, torch.int64).numpy()  # pinned: output then status words
    y, st = blk[:n].view(np.uint64), blk[n:].view(np.uint32)
    wsb = int(lib.fbm_lom_host_workspace(n, 1))
    ws = _host_workspace(wsb, dev)
    try:
        _call(lib.fbm_lom_protect_host, _np_ptr(x), N.FBM_F64, n, c, c2, tf, tm1, int(weight), _np_ptr(sec),
              _np_ptr(sg), len(secrets), 0, _np_ptr(nb), int(tau), 0, _np_ptr(y), _np_ptr(st), _ptr(ws), _stream())
    finally:
        _scrub_host_workspace(ws, wsb)
    _check_stats_host(st, n_nodes)
    if post is not None:
        raise post
    return y


def lom_aggregate_host(Y: np.ndarray, total_weight: int, clip=None, target=None) -> np.ndarray:
    """lom_aggregate of a HOST [P, n] uint64 matrix into host float64 averages, in one synchronous C call."""
    dev = device()
    lib = N.load()
    target = target or SAParameters.TARGET_RANGE
    if total_weight == 0:
        raise ZeroDivisionError("division by zero")
    if total_weight < 0 or total_weight > U64_MAX:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: total_sample_size must be in [1, 2^64) for the device path")
    negc, step = dequant_params(clip, target)
    Y = np.ascontiguousarray(Y)
    P, n = Y.shape
    blk = host_empty(n + N.STATS_WORDS // 2, torch.int64).numpy()  # pinned: averages then status words
    out, st = blk[:n].view(np.float64), blk[n:].view(np.uint32)
    wsb = int(lib.fbm_lom_host_workspace(n, P))
    ws = _host_workspace(wsb, dev)
    try:
        _call(lib.fbm_lom_aggregate_host, _np_ptr(Y), P, n, int(total_weight), negc, step, _np_ptr(out),
              _np_ptr(st), _ptr(ws), _stream())
    finally:
        _scrub_host_workspace(ws, wsb)
    _check_stats_host(st)
    return out


def prf_key(secret: bytes, nonce: bytes, tau: int, dev=None) -> bytes:
    dev = dev or device()
    sec = _secret_block([secret])
    nb = _nonce_block(nonce)
    if tau < 0:  # tau.to_bytes(16, 'big') (_lom.py:43-45)
        raise OverflowError("can't convert negative int to unsigned")
    if tau > U64_MAX:  # valid up to 2^128 in the reference; the device round counter is 64-bit
        raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: round counter {tau} >= 2^64 is outside "
                                          "the device path's domain")
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    _call(N.load().fbm_prf_key, _np_ptr(sec), _np_ptr(nb), int(tau), _ptr(out), _stream())
    return out.cpu().numpy().tobytes()


def lom_aggregate(Y: torch.Tensor, total_weight: int, clip=None, target=None,
                  want_out: bool = True, want_sums: bool = False):
    """Column sum (mod 2^64) + average + dequantise of a [P, n] int64 (u64) tensor."""
    dev = Y.device
    lib = N.load()
    target = target or SAParameters.TARGET_RANGE
    if total_weight == 0:
        raise ZeroDivisionError("division by zero")
    if total_weight < 0 or total_weight > U64_MAX:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: total_sample_size must be in [1, 2^64) for the device path")
    negc, step = dequant_params(clip, target)
    Y = Y.contiguous()
    P, n = Y.shape
    out = torch.empty(n, dtype=torch.float64, device=dev) if want_out else None
    sums = torch.empty(n, dtype=torch.int64, device=dev) if want_sums else None
    st = _stats(dev)
    _call(lib.fbm_lom_aggregate, _ptr(Y), P, n, int(total_weight), negc, step, _ptr(out), _ptr(sums), _ptr(st),
          _stream())
    _check_stats_or_defer(st)  # (inside deferred_checks: at its exit, e.g. the list aggregate's, after the D2H)
    return out, sums


def dequantize(u: torch.Tensor, clip=None, target=None) -> torch.Tensor:
    target = target or SAParameters.TARGET_RANGE
    negc, step = dequant_params(clip, target)
    u = u.contiguous()
    out = torch.empty(u.numel(), dtype=torch.float64, device=u.device)
    _call(N.load().fbm_dequantize, _ptr(u), u.numel(), negc, step, _ptr(out), _stream())
    return out


# ------------------------------------------------------------------------------------------
# Joye-Libert
# ------------------------------------------------------------------------------------------
def _biprime_limbs(biprime: int) -> np.ndarray:
    """N as 32 limbs.  Any 1 <= N < 2^1024: an odd N >= 3 runs on the Montgomery engines, an even one
    and N = 1 on the generic engine (csrc/fbm_gen.hip), as the reference computes with any N
    (_jls.py:37-73)."""
    if biprime < 1 or biprime.bit_length() > 1024:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: biprime must be an integer in [1, 2^1024) (the device path's domain)")
    return int_limbs(biprime, 32)


def _key_limbs(key: int) -> Tuple[np.ndarray, int]:
    if abs(key).bit_length() > 2048:
        raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: key larger than 2048 bits")
    return int_limbs(abs(key), 64), 1 if key < 0 else 0


JL_MAX_CT = 14_000_000  # include/fbm_secagg.h FBM_JL_MAX_CT: ciphertexts per library call

_ENGINES = {"auto": 0, "single": 1, "generic": 2, "triple": 3, "quad": 4}


class jl_engine:
    """Exponentiation engine for the JL calls this thread issues inside (the test build's per-thread
    policy, fbm_jl_set_engine in include/fbm_secagg_test.h; the block's calls run through the test
    build, _native.test_hooks): "auto" (the library's choice by launch size -- the product library's
    only policy), "single" (one lane per ciphertext: several concurrent launches that fill the chip
    together), "quad" / "triple" (four / three lanes per ciphertext: latency of a launch below the
    chip's lane count), "generic" (csrc/fbm_gen.hip, Barrett products for any modulus: even biprimes
    always take it; under this policy odd ones do too -- a cross-check of the Montgomery engines).
    Results are bit-identical under every engine; other threads are unaffected.

        with D.jl_engine("single"):
            ...  # the parties' concurrent encrypts
    """

    def __init__(self, mode: str):
        if mode not in _ENGINES:
            raise ValueError(f"engine must be one of {sorted(_ENGINES)}")
        self._mode, self._prev, self._hooks = _ENGINES[mode], None, N.test_hooks()

    def __enter__(self):
        self._hooks.__enter__()
        self._prev = N.load_test().fbm_jl_set_engine(self._mode)
        return self

    def __exit__(self, *exc):
        N.load_test().fbm_jl_set_engine(self._prev)
        return self._hooks.__exit__(*exc)


class jl_short:
    """The exponentiation's short path (binary chain with the 9-row short-base product, taken for a
    one-digest FDH h and N > 2^262) on or off for the JL calls this thread issues inside
    (the test build's fbm_jl_set_short; the block's calls run through the test build): off, every wave
    runs the sliding-window table path.  Results are bit-identical either way -- an A/B and test switch."""

    def __init__(self, on: bool):
        self._on, self._prev, self._hooks = 1 if on else 0, None, N.test_hooks()

    def __enter__(self):
        self._hooks.__enter__()
        self._prev = N.load_test().fbm_jl_set_short(self._on)
        return self

    def __exit__(self, *exc):
        N.load_test().fbm_jl_set_short(self._prev)
        return self._hooks.__exit__(*exc)


_clear_hooks = []  # callables run by jl_clear_caches (SecaggCrypter.drop_prepared registers itself)


def jl_clear_caches() -> None:
    """Drops what the process keeps between calls: the library's host-side caches
    (fbm_jl_clear_caches: the short path's constant C per (N, |key|) -- held under a SHA-256 digest
    of (N, |key|), never the key, and zeroed -- and the per-biprime public parameters), the
    synchronous host calls' device workspaces (zeroed), and any prepared factor of prepare_encrypt /
    prepare_aggregate (zeroed: with a node's ciphertext, its H(t_k)^key decrypts that node's update).
    The reference keeps nothing between calls (a fresh SecaggCrypter per call,
    fedbiomed/node/secagg/_secagg_round.py:142); call this after a round to do the same (the next call
    rebuilds C: a few ms of host arithmetic)."""
    N.load().fbm_jl_clear_caches()
    if N.TEST_LIB_PATH in N._libs:  # the test build keeps its own caches
        N._libs[N.TEST_LIB_PATH].fbm_jl_clear_caches()
    release_host_workspaces()
    for hook in list(_clear_hooks):
        hook()


def one_lane_round(dev=None) -> int:
    """Ciphertexts the one-lane engine holds resident at once: 64 lanes x 2 waves per SIMD x 4 SIMDs
    per CU x the device's CUs (131 072 on MI355X)."""
    if os.environ.get("FBM_ONE_LANE_ROUND"):  # (tests: stripes of the list API's overlapped encrypt)
        return max(1, int(os.environ["FBM_ONE_LANE_ROUND"]))
    dev = dev or device()
    return 512 * torch.cuda.get_device_properties(dev).multi_processor_count


def list_encrypt_stripes(n_ct: int, dev=None) -> List[Tuple[int, int]]:
    """Ciphertext stripes [c0, c1) of the list API's overlapped encrypt: one per full one-lane round,
    the partial round last (a single stripe below two rounds' worth: nothing to overlap there)."""
    r = one_lane_round(dev)
    if n_ct < 2 * r:
        return [(0, n_ct)]
    cuts = list(range(0, n_ct, r)) + [n_ct]
    if n_ct - cuts[-2] < r // 8:  # a sliver of a tail rides with the last full round
        cuts.pop(-2)
    return list(zip(cuts[:-1], cuts[1:]))


def jl_engine_for(n_ct: int) -> str:
    """The engine a launch of n_ct ciphertexts takes under this thread's policy (test build)."""
    return {1: "single", 2: "generic", 3: "triple", 4: "quad"}[N.load_test().fbm_jl_engine_for(int(n_ct))]


def lom_aggregate_kernel(n_parties: int, y: torch.Tensor) -> str:
    """The LOM aggregate kernel a launch over y ([n_parties, n] in HBM) takes, as rocprofv3 names it
    without the "fbm::" namespace (test build, fbm_test_lom_aggregate_kernel)."""
    buf = ctypes.create_string_buffer(128)
    _call(N.load_test().fbm_test_lom_aggregate_kernel, int(n_parties), int(y.shape[-1]), _ptr(y), buf, len(buf))
    return buf.value.decode()


def jl_chunk_ct() -> int:
    """Ciphertexts per library call (FBM_JL_CHUNK_CT lowers it, for tests of the striping)."""
    v = int(os.environ.get("FBM_JL_CHUNK_CT", JL_MAX_CT))
    return max(1, min(v, JL_MAX_CT))


class jl_exp_batch:
    """Within this context the JL exponentiations of PendingEncrypt.finish() (non-negative key)
    and PendingFactor.exponentiate() are recorded, not launched; at exit ONE launch runs them all
    on the current stream (fbm_jl_batch_begin / fbm_jl_batch_flush): one chunk counter over every
    party's ciphertexts, so the chip's rounds pack whatever the parts' sizes and however the
    streams map onto the hardware queues.  The recorded calls' prologues must be complete on the
    current stream at exit (wait on their streams first) and their outputs are valid after it;
    the same biprime throughout; at most 24 calls.  If the block raises, the batch is dropped: the
    recorded exponentiations never run, and finish() on any of their Pending objects raises
    instead of returning unwritten memory.  A factor's inverse (PendingFactor.finish)
    goes after the context.  An even biprime's calls (the generic engine) are not recorded: they
    launch when issued, on the current stream.

        with D.jl_exp_batch():
            cts = [pend[p].finish() for p in range(P)]
            pf.exponentiate()
        factor = pf.finish()
    """

    _tls = threading.local()

    def __init__(self, dev=None):
        self._dev, self._keep, self._recorded = dev, [], []

    @staticmethod
    def active() -> Optional["jl_exp_batch"]:
        return getattr(jl_exp_batch._tls, "cur", None)

    def keep(self, tensors) -> None:
        """device tensors a recorded call reads or writes (kept alive until the launch, then
        marked as used on the launch stream for the caching allocator)"""
        self._keep += [t for t in tensors if isinstance(t, torch.Tensor) and t.is_cuda]

    def record(self, pending) -> None:
        """a Pending object whose exponentiation this batch recorded (invalidated on abort)"""
        self._recorded.append(pending)

    def __enter__(self):
        if jl_exp_batch.active() is not None:
            raise RuntimeError("jl_exp_batch contexts do not nest")
        _call(N.load().fbm_jl_batch_begin)
        jl_exp_batch._tls.cur = self
        return self

    def __exit__(self, exc_type, exc, tb):
        jl_exp_batch._tls.cur = None
        lib = N.load()
        if exc_type is not None:
            lib.fbm_jl_batch_abort()
            for p in self._recorded:  # their exponentiations never ran
                p._aborted = True
            self._recorded, self._keep = [], []
            return False
        ws = torch.empty(int(lib.fbm_jl_batch_workspace()), dtype=torch.uint8, device=self._dev or device())
        _call(lib.fbm_jl_batch_flush, _ptr(ws), ws.numel(), _stream())
        cur = torch.cuda.current_stream(ws.device)
        for t in self._keep:
            t.record_stream(cur)
        self._keep = []
        return False


class PendingEncrypt:
    """A JL encrypt whose prologue kernels are issued and whose exponentiation is not yet
    (jl_encrypt(..., defer_exp=True)); finish() issues it on the current stream and returns
    the ciphertext tensor (inside a jl_exp_batch: records it for the batch's launch).  Holds
    the workspace and the status word until then."""

    def __init__(self, args, ct, ws, st):
        self._args, self._ct, self._ws, self._st, self._aborted = args, ct, ws, st, False

    def finish(self) -> torch.Tensor:
        if self._aborted:
            raise RuntimeError("this encrypt's exponentiation was recorded in a jl_exp_batch that was aborted: "
                               "its ciphertexts were never computed")
        if self._args is not None:
            lib = N.load()
            n0 = lib.fbm_jl_batch_count()
            _call(lib.fbm_jl_encrypt_phase, *self._args, _stream(), 2)
            b = jl_exp_batch.active()
            if b is not None:
                b.keep([self._ct, *self._ws])
                if lib.fbm_jl_batch_count() > n0:
                    b.record(self)
            _check_stats_or_defer(self._st)
            self._args = None
        return self._ct


JL_ROUND_BITS = 8192  # FDH.H's int(t).to_bytes(1024, 'big') of t = (k << 512) | tau


def _check_round(tau: int) -> np.ndarray:
    """The JL round -> its N.TAU_LIMBS limbs for the C-ABI (ABI 3: any round the reference hashes).
    FDH.H serialises t = (k << 512) | tau with int(t).to_bytes(1024, 'big') (_jls.py:451-467, 744-748):
    a negative round, or one of 2^8192 or more, is the reference's OverflowError there."""
    tau = operator.index(tau)
    if tau < 0:
        raise OverflowError("can't convert negative int to unsigned")
    if tau >> JL_ROUND_BITS:
        raise OverflowError("int too big to convert")
    if tau >> 512 and N.loaded_abi is not None and N.loaded_abi < 3:
        # an ABI 2 A/B variant (FBM_AB_VARIANT=1) reads 16 of the round's limbs: it would hash tau mod 2^512
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: the loaded library (ABI {N.loaded_abi}) hashes rounds below 2^512 only")
    return int_limbs(tau, N.TAU_LIMBS)


def jl_encrypt(x: torch.Tensor, biprime: int, key: int, tau: int, n_users: int, clip=None, target=None,
               weight: int = 1, slot: Optional[Tuple[int, int]] = None, ct_offset: int = 0,
               defer_exp: bool = False, kind: Optional[str] = None, out: Optional[torch.Tensor] = None,
               factor: Optional[torch.Tensor] = None):
    """One party's JL ciphertexts as an int32 [n_ct, 64] tensor of 32-bit limbs.
    `factor`: this party's H(t_k)^key for these ciphertexts computed ahead (jl_decrypt_factor with the
    party's key, round and ct_offset): the encrypt is then (N pt + 1) F mod N^2 (fbm_jl_encrypt_factor),
    bit for bit the exponentiation's; odd N >= 3 only.
    `out`: a contiguous int32 [n_ct, 64] device tensor to write them into (e.g. this party's row of the
    [P, n_ct, 64] block the aggregate takes), returned instead of a new one.
    `slot` overrides the (element_size, comp_ratio) packing.  `kind` selects a raw input:
    "u128" = int64 [n, 2] (lo, hi) integers packed into the VES slots (JoyeLibert.protect),
    "pt" = int32 [n, 32] plaintext limbs encrypted as they are (UserKey.encrypt; slot (1, 1)).
    defer_exp: issue only the prologue and return a PendingEncrypt (one library call's worth of
    ciphertexts at most)."""
    dev = x.device
    lib = N.load()
    target = target or SAParameters.TARGET_RANGE
    es, cr = slot if slot else jl_slot(target, n_users)
    raw = kind is not None or x.dtype == torch.int64
    c, c2, tf, tm1 = (1.0, 2.0, 1.0, 0) if raw else quant_params(clip, target)
    tl = _check_round(tau)
    x = x.contiguous()
    if kind == "u128":
        xdt, n = N.FBM_U128, x.shape[0]
    elif kind == "pt":
        xdt, n, es, cr = N.FBM_PT, x.shape[0], 1, 1
    elif kind is None:
        xdt, n = _x_dtype(x), x.numel()
    else:
        raise ValueError(f"unknown input kind {kind!r}")
    n_ct = (n + cr - 1) // cr
    if out is None:
        ct = torch.empty((n_ct, 64), dtype=torch.int32, device=dev)
    else:
        if (out.dtype != torch.int32 or tuple(out.shape) != (n_ct, 64) or not out.is_contiguous()
                or out.device != dev):
            raise ValueError(f"out must be a contiguous int32 ({n_ct}, 64) tensor on {dev}, got "
                             f"{out.dtype} {tuple(out.shape)} on {out.device}")
        ct = out
    if n_ct == 0:
        return ct
    bp = _biprime_limbs(biprime)
    kl, kneg = _key_limbs(key)
    chunk = jl_chunk_ct()  # calls above the library's per-call cap run as ct_offset stripes
    ws = torch.empty(int(lib.fbm_jl_encrypt_workspace(min(n_ct, chunk))), dtype=torch.uint8, device=dev)
    if factor is not None:
        if defer_exp:
            raise ValueError("an encrypt with its factor computed ahead has no exponentiation to defer")
        if (factor.dtype != torch.int32 or tuple(factor.shape) != (n_ct, 64) or not factor.is_contiguous()
                or factor.device != dev):
            raise ValueError(f"factor must be the contiguous int32 ({n_ct}, 64) H(t_k)^key of these ciphertexts "
                             f"on {dev}")
        for k0 in range(0, n_ct, chunk):
            k1 = min(n_ct, k0 + chunk)
            xs = x[k0 * cr:min(n, k1 * cr)]
            st = _stats(dev)
            _call(lib.fbm_jl_encrypt_factor, _ptr(xs), xdt, xs.shape[0] if kind else xs.numel(), c, c2, tf, tm1,
                  int(weight) & U64_MAX, es, cr, _np_ptr(bp), _ptr(factor[k0:k1]), _ptr(ct[k0:k1]), _ptr(ws),
                  _ptr(st), _stream())
            _check_stats_or_defer(st)
        return ct
    if defer_exp:
        if n_ct > chunk:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value}: a deferred encrypt takes at most {chunk} ciphertexts")
        st = _stats(dev)
        args = (_ptr(x), xdt, n, c, c2, tf, tm1, int(weight) & U64_MAX, es, cr, _np_ptr(bp), _np_ptr(kl), kneg,
                _np_ptr(tl), int(ct_offset), _ptr(ct), _ptr(ws), _ptr(st))
        _call(lib.fbm_jl_encrypt_phase, *args, _stream(), 1)
        return PendingEncrypt(args, ct, (ws, x, bp, kl, tl), st)
    for k0 in range(0, n_ct, chunk):
        k1 = min(n_ct, k0 + chunk)
        xs = x[k0 * cr:min(n, k1 * cr)]
        st = _stats(dev)  # one status word per call (each call zeroes its own)
        _call(lib.fbm_jl_encrypt, _ptr(xs), xdt, xs.shape[0] if kind else xs.numel(), c, c2, tf, tm1,
              int(weight) & U64_MAX, es, cr,
              _np_ptr(bp), _np_ptr(kl), kneg, _np_ptr(tl), int(ct_offset) + k0, _ptr(ct[k0:k1]), _ptr(ws), _ptr(st),
              _stream())
        _check_stats_or_defer(st)
    return ct


class PendingFactor:
    """A decryption factor issued phase by phase (jl_decrypt_factor(..., phased=True) issues
    constants + FDH): exponentiate() and then finish() (the inverse of a negative key) issue the
    rest on the current stream; finish() returns the factor tensor."""

    def __init__(self, args, f, keep, st):
        self._args, self._f, self._keep, self._st, self._done, self._aborted = args, f, keep, st, 1, False

    def _phase(self, bit):
        if self._aborted:
            raise RuntimeError("this decryption factor's exponentiation was recorded in a jl_exp_batch that was "
                               "aborted: the factor was never computed")
        if not self._done & bit:
            lib = N.load()
            n0 = lib.fbm_jl_batch_count()
            _call(lib.fbm_jl_decrypt_factor_phase, *self._args, _stream(), bit)
            self._done |= bit
            b = jl_exp_batch.active()
            if b is not None:
                b.keep([self._f, *self._keep])
                if lib.fbm_jl_batch_count() > n0:
                    b.record(self)

    def exponentiate(self) -> "PendingFactor":
        self._phase(2)
        return self

    def finish(self) -> torch.Tensor:
        self._phase(2)
        if not self._done & 4:
            self._phase(4)
            _check_stats_or_defer(self._st)
        return self._f


def jl_decrypt_factor(n_ct: int, biprime: int, key: int, tau: int, ct_offset: int = 0, dev=None,
                      phased: bool = False):
    """ServerKey's H(t_k)^key mod N^2 for ciphertexts [ct_offset, ct_offset + n_ct) of round
    `tau` as int32 [n_ct, 64] limbs -- needs no ciphertext, so it can run while parties encrypt.
    phased: issue only the first phase (constants + FDH) and return a PendingFactor."""
    dev = dev or device()
    lib = N.load()
    tl = _check_round(tau)
    f = torch.empty((n_ct, 64), dtype=torch.int32, device=dev)
    if n_ct == 0:
        return f
    bp = _biprime_limbs(biprime)
    kl, kneg = _key_limbs(key)
    chunk = jl_chunk_ct()
    ws = torch.empty(int(lib.fbm_jl_aggregate_workspace(min(n_ct, chunk))), dtype=torch.uint8, device=dev)
    if phased:
        if n_ct > chunk:
            raise FedbiomedSecaggCrypterError(
                f"{ErrorNumbers.FB624.value}: a phased decryption factor takes at most {chunk} ciphertexts")
        st = _stats(dev)
        args = (n_ct, _np_ptr(bp), _np_ptr(kl), kneg, _np_ptr(tl), int(ct_offset), _ptr(f), _ptr(ws), _ptr(st))
        _call(lib.fbm_jl_decrypt_factor_phase, *args, _stream(), 1)
        return PendingFactor(args, f, (ws, bp, kl, tl), st)
    for k0 in range(0, n_ct, chunk):
        k1 = min(n_ct, k0 + chunk)
        st = _stats(dev)
        _call(lib.fbm_jl_decrypt_factor, k1 - k0, _np_ptr(bp), _np_ptr(kl), kneg, _np_ptr(tl), int(ct_offset) + k0,
              _ptr(f[k0:k1]), _ptr(ws), _ptr(st), _stream())
        _check_stats_or_defer(st)
    return f


def jl_aggregate(cts: torch.Tensor, biprime: int, key: int, tau: int, n_expected: int, total_weight: int,
                 clip=None, target=None, want_out: bool = True, want_sums: bool = False,
                 slot: Optional[Tuple[int, int]] = None, ct_offset: int = 0, factor: Optional[torch.Tensor] = None):
    """Aggregate [P, n_ct, 64] int32 ciphertext limbs -> (float64 [n_out], int64 [n_out, 2] sums).
    `factor`: the round's precomputed jl_decrypt_factor (same key, tau, ct range), or None."""
    dev = cts.device
    lib = N.load()
    target = target or SAParameters.TARGET_RANGE
    P, n_ct, _ = cts.shape
    es, cr = slot if slot else jl_slot(target, P)
    n_out = max(0, min(int(n_expected), n_ct * cr))
    negc, step = dequant_params(clip, target)
    if total_weight == 0:
        raise ZeroDivisionError("division by zero")
    if total_weight < 0 or total_weight > U64_MAX:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: total_sample_size must be in [1, 2^64) for the device path")
    tl = _check_round(tau) if factor is None else None  # a given factor fixes the round already
    out = torch.empty(n_out, dtype=torch.float64, device=dev) if want_out else None
    sums = torch.empty((n_out, 2), dtype=torch.int64, device=dev) if want_sums else None
    if n_ct == 0:
        return out, sums
    if factor is not None:
        factor = factor.contiguous()
        if factor.dtype != torch.int32 or tuple(factor.shape) != (n_ct, 64) or factor.device != dev:
            raise ValueError("factor must be the int32 [n_ct, 64] jl_decrypt_factor of these ciphertexts")
    bp = _biprime_limbs(biprime)
    kl, kneg = _key_limbs(key)
    chunk = jl_chunk_ct()
    cts = cts.contiguous()
    ws = torch.empty(int(lib.fbm_jl_aggregate_workspace(min(n_ct, chunk))), dtype=torch.uint8, device=dev)
    for k0 in range(0, n_ct, chunk):
        k1 = min(n_ct, k0 + chunk)
        part = cts[:, k0:k1].contiguous() if (k0, k1) != (0, n_ct) else cts
        e0, e1 = k0 * cr, min(n_out, k1 * cr)
        if e1 <= e0:
            break
        st = _stats(dev)
        o, sm = _ptr(out[e0:e1] if want_out else None), _ptr(sums[e0:e1] if want_sums else None)
        if factor is None:
            _call(lib.fbm_jl_aggregate, _ptr(part), P, k1 - k0, es, cr, e1 - e0, _np_ptr(bp), _np_ptr(kl), kneg,
                  _np_ptr(tl), int(ct_offset) + k0, int(total_weight), negc, step, o, sm, _ptr(ws), _ptr(st), _stream())
        else:
            _call(lib.fbm_jl_aggregate_factor, _ptr(part), P, k1 - k0, es, cr, e1 - e0, _np_ptr(bp),
                  _ptr(factor[k0:k1]), int(total_weight), negc, step, o, sm, _ptr(ws), _ptr(st), _stream())
        _check_stats_or_defer(st)  # (inside deferred_checks: at its exit, e.g. the list aggregate's stripes)
    return out, sums


# ------------------------------------------------------------------------------------------
# the JoyeLibert object API (secagg/_jls.py): VES, FDH, ciphertext products, raw decryption
# ------------------------------------------------------------------------------------------
def ints_to_u128(values: Sequence[int], dev=None) -> torch.Tensor:
    """list of ints in [0, 2^128) -> int64 [n, 2] (lo, hi) device tensor; FB624 outside."""
    vals = values if isinstance(values, list) else list(values)
    host = host_empty((len(vals), 2), torch.int64)
    bad = _pyconv().ints_to_bytes(vals, 16, host.numpy()) if vals else -1
    if bad >= 0:
        v = vals[bad]
        if not isinstance(v, int):
            try:
                v = v.__index__()
            except (AttributeError, TypeError):
                raise TypeError(f"expected integers, got {type(vals[bad])}") from None
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: integer {v} outside [0, 2^128), the device path's domain")
    return host.to(dev or device())


def u128_to_ints(t: torch.Tensor) -> List[int]:
    a = to_host(t).numpy().view(np.uint64)
    return [int(lo) | (int(hi) << 64) for lo, hi in a.tolist()]


def ints_to_pt(values: Sequence[int], modulus: int, dev=None) -> torch.Tensor:
    """Plaintext ints -> int32 [n, 32] limbs; values outside [0, 2^1024) are replaced by their
    residue mod N (N*pt + 1 mod N^2 depends on pt mod N only)."""
    vals = values if isinstance(values, list) else list(values)
    host = host_empty((len(vals), 32), torch.int32)
    buf = host.numpy()
    bad = _pyconv().ints_to_bytes(vals, 128, buf) if vals else -1
    while bad >= 0:
        v = operator.index(vals[bad]) % modulus
        buf[bad] = np.frombuffer(v.to_bytes(128, "little"), dtype=np.int32)
        rest = _pyconv().ints_to_bytes(vals[bad + 1:], 128, buf[bad + 1:])
        bad = -1 if rest < 0 else bad + 1 + rest
    return host.to(dev or device())


def int_multiply(vals: torch.Tensor, k: int) -> List[int]:
    """[v * k] (utils.multiply, _secagg_utils.py:122-134) on the device for int64 [n, 2] (lo, hi) values
    v < 2^128 and an integer k with |k| < 2^64: the exact products (< 2^192), negative for k < 0 as in
    the reference; FB624 for a wider k."""
    k = operator.index(k)
    if abs(k) > U64_MAX:
        raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: factor {k} outside (-2^64, 2^64), "
                                          "the device path's domain")
    out = torch.empty((vals.shape[0], 3), dtype=torch.int64, device=vals.device)
    st = _stats(vals.device)
    _call(N.load().fbm_int_ops, _ptr(vals.contiguous()), vals.shape[0], abs(k), 0, _ptr(out), _ptr(st), _stream())
    w = to_host(out).numpy().view(np.uint64)
    sign = -1 if k < 0 else 1
    return [sign * (int(a) | (int(b) << 64) | (int(c) << 128)) for a, b, c in w.tolist()]


def int_true_divide(vals: torch.Tensor, k) -> List[float]:
    """[v / k] (utils.divide, _secagg_utils.py:137-149) on the device for v < 2^128: an integer k of any
    size with Python's correctly rounded int/int true division (|k| >= 2^64: fbm_int_true_div_big), a
    real k with Python's int / float (float(v), then the IEEE division); the divisor is never truncated.
    k == 0 raises the reference's ZeroDivisionError."""
    import numbers

    if isinstance(k, numbers.Integral):
        k = operator.index(k)
        if k == 0:
            raise ZeroDivisionError("division by zero")
        if abs(k) > U64_MAX:
            out = torch.empty(vals.shape[0], dtype=torch.float64, device=vals.device)
            kw = max(1, (abs(k).bit_length() + 31) // 32)
            _call(N.load().fbm_int_true_div_big, _ptr(vals.contiguous()), vals.shape[0], _np_ptr(int_limbs(abs(k), kw)),
                  kw, 1 if k < 0 else 0, _ptr(out), _stream())
            return to_host(out).numpy().tolist()
        op, karg = (1 if k > 0 else 3), abs(k)
    elif isinstance(k, numbers.Real):
        kd = float(k)
        if kd == 0.0:
            raise ZeroDivisionError("float division by zero")
        op, karg = 2, int(np.frombuffer(np.float64(kd).tobytes(), dtype=np.uint64)[0])
    else:
        raise TypeError(f"unsupported operand type(s) for /: 'int' and '{type(k).__name__}'")
    out = torch.empty(vals.shape[0], dtype=torch.float64, device=vals.device)
    st = _stats(vals.device)
    _call(N.load().fbm_int_ops, _ptr(vals.contiguous()), vals.shape[0], karg, op, _ptr(out), _ptr(st), _stream())
    return to_host(out).numpy().tolist()


def jl_pack(vals: torch.Tensor, es: int, cr: int) -> torch.Tensor:
    """VES.encode on the device: int64 [n, 2] (lo, hi) values -> int32 [ceil(n/cr), 32] limbs."""
    n = vals.shape[0]
    pt = torch.empty(((n + cr - 1) // cr, 32), dtype=torch.int32, device=vals.device)
    st = _stats(vals.device)
    _call(N.load().fbm_jl_pack, _ptr(vals.contiguous()), N.FBM_U128, n, int(es), int(cr), _ptr(pt), _ptr(st),
          _stream())
    _check_stats(st)
    return pt


def _rows_of(vals: List[int], w: int) -> np.ndarray:
    out = np.zeros((len(vals), w), dtype=np.uint32)
    for i, v in enumerate(vals):
        out[i] = int_limbs(v, w)
    return out


def ves_pack_any(V: List[int], es: int, cr: int, dev=None) -> List[int]:
    """VES.encode of any shape (fbm_ves_pack): ints of any width and sign, slots of any es, plaintexts of
    any width; the reference's OR packing (_jls.py:118-144, 169-176).  With a negative value the rows go
    to the device in two's complement (one sign bit above the widest value) and its sign extends to the top
    of its plaintext, which comes back as Python's negative OR: the pw-word pattern minus 2^(32 pw)."""
    dev = dev or device()
    if not V:
        return []
    signed = min(V) < 0
    if signed and (N.loaded_abi or 0) < 4:
        raise FedbiomedSecaggCrypterError(
            f"{ErrorNumbers.FB624.value}: VES.encode of negative values needs an ABI 4 library (loaded: "
            f"ABI {N.loaded_abi})")
    wv = max(1, (max(v.bit_length() for v in V) + (1 if signed else 0) + 31) // 32)
    pw = (es * (cr - 1) + 32 * wv + 31) // 32
    n_ct = (len(V) + cr - 1) // cr
    rows = [v & ((1 << (32 * wv)) - 1) for v in V] if signed else V  # two's complement rows
    x = torch.from_numpy(_rows_of(rows, wv).view(np.int32)).to(dev)
    pt = torch.empty((n_ct, pw), dtype=torch.int32, device=dev)
    _call(N.load().fbm_ves_pack, _ptr(x), len(V), wv, es, cr, pw, 1 if signed else 0, _ptr(pt), _stream())
    out = limbs_to_ints_w(pt, pw)
    if signed:
        top, full = 1 << (32 * pw - 1), 1 << (32 * pw)
        out = [e - full if e & top else e for e in out]
    return out


def ves_unpack_any(E: List[int], es: int, cr: int, v_expected: int, dev=None) -> List[int]:
    """VES.decode of any shape (fbm_ves_unpack): slot j of each plaintext, (e >> es j) & (2^es - 1), for
    min(remaining, cr) slots per plaintext (_jls.py:146-167, 179-192); only the low es cr bits of a plaintext
    are read -- a negative one's two's complement, as Python's shifts and masks see it."""
    dev = dev or device()
    n_out = min(int(v_expected), len(E) * cr)
    if n_out <= 0:
        return []
    pw = (es * cr + 31) // 32
    ow = (es + 31) // 32
    pts = torch.from_numpy(_rows_of([int(e) & ((1 << (32 * pw)) - 1) for e in E], pw).view(np.int32)).to(dev)
    vals = torch.empty((n_out, ow), dtype=torch.int32, device=dev)
    _call(N.load().fbm_ves_unpack, _ptr(pts), len(E), pw, es, cr, n_out, ow, _ptr(vals), _stream())
    return limbs_to_ints_w(vals, ow)


def jl_unpack(pt: torch.Tensor, es: int, cr: int, n_out: int) -> torch.Tensor:
    """VES.decode on the device: int32 [n_ct, 32] limbs -> int64 [n_out, 2] (lo, hi) slot values."""
    n_ct = pt.shape[0]
    n_out = max(0, min(int(n_out), n_ct * cr))
    vals = torch.empty((n_out, 2), dtype=torch.int64, device=pt.device)
    if n_out:
        _call(N.load().fbm_jl_unpack, _ptr(pt.contiguous()), n_ct, int(es), int(cr), n_out, _ptr(vals), _stream())
    return vals


def fdh_modulus(m: int) -> Tuple[int, bool]:
    """FDH gcd modulus M -> (odd part of M or of its square root, M even): gcd(r, M) == 1 iff r
    is coprime to that odd part (and odd, for an even M).  FB624 outside the device domain."""
    m = operator.index(m)
    if m > 0:
        root = math.isqrt(m)
        base = root if root * root == m else m
        even = base % 2 == 0
        while base and base % 2 == 0:
            base //= 2
        if 1 <= base < 2**1024:
            return base, even
    raise FedbiomedSecaggCrypterError(
        f"{ErrorNumbers.FB624.value}: FDH modulus outside the device path's domain (odd part of M or of its "
        "square root in [1, 2^1024))")


def jl_fdh(n_ct: int, modulus: int, tau: int, ct_offset: int = 0, dev=None) -> torch.Tensor:
    """FDH.H(t_k) of t_k = ((k + ct_offset) << 512) | tau, bits_size 2048, gcd against `modulus`
    (any M: its odd part, or its square root's) -> int32 [n_ct, 64] limbs."""
    dev = dev or device()
    tl = _check_round(tau)
    if not (0 <= ct_offset and ct_offset + max(n_ct, 1) - 1 <= U64_MAX):
        raise FedbiomedSecaggCrypterError(f"{ErrorNumbers.FB624.value}: FDH input outside the device path's domain")
    odd, even = fdh_modulus(modulus)
    h = torch.empty((n_ct, 64), dtype=torch.int32, device=dev)
    st = _stats(dev)
    ol = int_limbs(odd, 32)
    _call(N.load().fbm_jl_fdh, n_ct, _np_ptr(ol), 1 if even else 0, _np_ptr(tl), int(ct_offset),
          _ptr(h), _ptr(st), _stream())
    _check_stats(st)
    return h


def jl_fdh_msg(ts: List[int], bits_size: int, modulus: int, dev=None) -> torch.Tensor:
    """FDH(bits_size, modulus).H(t) for each t (any bits_size; fbm_jl_fdh_msg) -> int32 [len(ts), hw] limbs
    (hw = fbm_jl_fdh_msg_row_words(bits_size): 128, or 8 per digest when r may take 16 .. 255 digests).
    The reference's to_bytes errors are raised here first: t < 0 and t >= 2^(8 (bits_size // 2))."""
    L = bits_size // 2
    if L < 0:
        raise ValueError("length argument must be non-negative")
    for t in ts:
        if t < 0:
            raise OverflowError("can't convert negative int to unsigned")
        if t.bit_length() > 8 * L:
            raise OverflowError("int too big to convert")
    dev = dev or device()
    tw = max(1, (L + 3) // 4)
    host = np.zeros((len(ts), tw), dtype=np.uint32)
    for i, t in enumerate(ts):
        host[i] = int_limbs(t, tw)
    odd, even = fdh_modulus(modulus)
    lib = N.load()
    hw = int(lib.fbm_jl_fdh_msg_row_words(int(bits_size)))  # 128, or 8 per digest past 15 (ABI 4)
    h = torch.empty((len(ts), hw), dtype=torch.int32, device=dev)
    st = _stats(dev)
    t_dev = torch.from_numpy(host.view(np.int32)).to(dev)
    _call(lib.fbm_jl_fdh_msg, len(ts), _ptr(t_dev), tw, int(bits_size), _np_ptr(int_limbs(odd, 32)),
          1 if even else 0, _ptr(h), hw, _ptr(st), _stream())
    _check_stats(st)
    return h


def jl_product(cts: torch.Tensor, biprime: int) -> torch.Tensor:
    """prod_u cts[u] mod N^2 (EncryptedNumber sums): int32 [P, n_ct, 64] -> [n_ct, 64], canonical."""
    P, n_ct, _ = cts.shape
    out = torch.empty((n_ct, 64), dtype=torch.int32, device=cts.device)
    if n_ct == 0:
        return out
    lib = N.load()
    bp = _biprime_limbs(biprime)
    ws = torch.empty(int(lib.fbm_jl_aggregate_workspace(n_ct)), dtype=torch.uint8, device=cts.device)
    _call(lib.fbm_jl_product, _ptr(cts.contiguous()), P, n_ct, _np_ptr(bp), _ptr(out), _ptr(ws), _stream())
    return out


def jl_decrypt(cts: torch.Tensor, biprime: int, key: int, tau: int, ct_offset: int = 0) -> torch.Tensor:
    """ServerKey.decrypt (delta = 1) of the product of P ciphertext rows: int32 [P, n_ct, 64] ->
    x = ((prod * H(t_k)^key mod N^2) - 1) // N mod N as int32 [n_ct, 32] limbs."""
    P, n_ct, _ = cts.shape
    dev = cts.device
    x = torch.empty((n_ct, 32), dtype=torch.int32, device=dev)
    if n_ct == 0:
        return x
    tl = _check_round(tau)
    lib = N.load()
    bp = _biprime_limbs(biprime)
    kl, kneg = _key_limbs(key)
    ws = torch.empty(int(lib.fbm_jl_aggregate_workspace(n_ct)), dtype=torch.uint8, device=dev)
    st = _stats(dev)
    _call(lib.fbm_jl_decrypt, _ptr(cts.contiguous()), P, n_ct, _np_ptr(bp), _np_ptr(kl), kneg, _np_ptr(tl),
          int(ct_offset), _ptr(x), _ptr(ws), _ptr(st), _stream())
    _check_stats(st)
    return x


def jl_powmod(h: torch.Tensor, biprime: int, key: int, pt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Caller-given bases (the hashes of a PublicParam whose hashing function is not FBM's FDH):
    (N pt[k] + 1) h[k]^key mod N^2 with pt (int32 [n_ct, 32] plaintext limbs, UserKey.encrypt), or
    h[k]^key mod N^2 without (ServerKey.decrypt's powmod), as int32 [n_ct, 64] limbs; h: int32 [n_ct, 64]
    limbs (< 2^2048).  A negative key inverts first: a base without an inverse is ZeroDivisionError."""
    n_ct = h.shape[0]
    dev = h.device
    out = torch.empty((n_ct, 64), dtype=torch.int32, device=dev)
    if n_ct == 0:
        return out
    lib = N.load()
    bp = _biprime_limbs(biprime)
    kl, kneg = _key_limbs(key)
    h = h.contiguous()
    pt = pt.contiguous() if pt is not None else None
    chunk = jl_chunk_ct()
    ws = torch.empty(int(lib.fbm_jl_encrypt_workspace(min(n_ct, chunk))), dtype=torch.uint8, device=dev)
    for k0 in range(0, n_ct, chunk):
        k1 = min(n_ct, k0 + chunk)
        st = _stats(dev)
        _call(lib.fbm_jl_powmod, _ptr(h[k0:k1]), _ptr(pt[k0:k1] if pt is not None else None), k1 - k0, _np_ptr(bp),
              _np_ptr(kl), kneg, _ptr(out[k0:k1]), _ptr(ws), _ptr(st), _stream())
        _check_stats(st)
    return out


def jl_decrypt_with(cts: torch.Tensor, biprime: int, factor: torch.Tensor) -> torch.Tensor:
    """ServerKey.decrypt's x = ((prod_u cts[u] * factor mod N^2) - 1) // N mod N for a jl_powmod factor:
    int32 [P, n_ct, 64] ciphertext limbs -> int32 [n_ct, 32]."""
    P, n_ct, _ = cts.shape
    dev = cts.device
    x = torch.empty((n_ct, 32), dtype=torch.int32, device=dev)
    if n_ct == 0:
        return x
    factor = factor.contiguous()
    if factor.dtype != torch.int32 or tuple(factor.shape) != (n_ct, 64) or factor.device != dev:
        raise ValueError("factor must be the int32 [n_ct, 64] jl_powmod power of these ciphertexts' bases")
    lib = N.load()
    bp = _biprime_limbs(biprime)
    ws = torch.empty(int(lib.fbm_jl_aggregate_workspace(n_ct)), dtype=torch.uint8, device=dev)
    st = _stats(dev)
    _call(lib.fbm_jl_decrypt_with, _ptr(cts.contiguous()), P, n_ct, _np_ptr(bp), _ptr(factor), _ptr(x), _ptr(ws),
          _ptr(st), _stream())
    _check_stats(st)
    return x


# ------------------------------------------------------------------------------------------
# additive secret sharing (secagg/_additive_ss.py)
# ------------------------------------------------------------------------------------------
I64_MIN, U64_LIM = -(2**63), 2**64


def ass_split(secret: torch.Tensor, n_shares: int, bit_length: Optional[int] = None, unsigned: bool = False,
              seed: Optional[bytes] = None, nonce: Optional[bytes] = None, elem_offset: int = 0) -> torch.Tensor:
    """Device int64 vector (uint64 bit patterns if `unsigned`) -> int64 [n_shares, n, 2]
    int128 shares (lo, hi).  `seed` (32 B) / `nonce` (8 B) default to fresh OS randomness."""
    import secrets as _secrets

    lib = N.load()
    secret = secret.contiguous()
    n = secret.numel()
    shares = torch.empty((n_shares, n, 2), dtype=torch.int64, device=secret.device)
    seed = seed if seed is not None else _secrets.token_bytes(32)
    nonce = nonce if nonce is not None else _secrets.token_bytes(8)
    if len(seed) != 32 or len(nonce) != 8:
        raise ValueError("seed must be 32 bytes and nonce 8 bytes")
    sb = np.frombuffer(seed, dtype=np.uint8).copy()
    nb = np.frombuffer(nonce, dtype=np.uint8).copy()
    _call(lib.fbm_ass_split, _ptr(secret), N.FBM_U64 if unsigned else N.FBM_I64, n, int(n_shares),
          -1 if bit_length is None else int(bit_length), _np_ptr(sb), _np_ptr(nb), int(elem_offset), _ptr(shares),
          _stream())
    return shares


def ass_reconstruct(shares: torch.Tensor) -> torch.Tensor:
    """int64 [P, n, 2] int128 shares -> int64 [n, 2] int128 exact column sum."""
    lib = N.load()
    shares = shares.contiguous()
    P, n, _ = shares.shape
    out = torch.empty((n, 2), dtype=torch.int64, device=shares.device)
    _call(lib.fbm_ass_reconstruct, _ptr(shares), int(P), n, _ptr(out), _stream())
    return out


def ass_split_wide(secret: torch.Tensor, n_shares: int, l_out: int, bit_length: Optional[int] = None,
                   seed: Optional[bytes] = None, nonce: Optional[bytes] = None, elem_offset: int = 0) -> torch.Tensor:
    """int32 [l_in, n] two's-complement limbs (limb-major) -> int32 [n_shares, l_out, n] shares."""
    import secrets as _secrets

    lib = N.load()
    secret = secret.contiguous()
    l_in, n = secret.shape
    shares = torch.empty((n_shares, l_out, n), dtype=torch.int32, device=secret.device)
    seed = seed if seed is not None else _secrets.token_bytes(32)
    nonce = nonce if nonce is not None else _secrets.token_bytes(8)
    if len(seed) != 32 or len(nonce) != 8:
        raise ValueError("seed must be 32 bytes and nonce 8 bytes")
    sb = np.frombuffer(seed, dtype=np.uint8).copy()
    nb = np.frombuffer(nonce, dtype=np.uint8).copy()
    _call(lib.fbm_ass_split_wide, _ptr(secret), n, int(l_in), int(n_shares),
          -1 if bit_length is None else int(bit_length), int(l_out), _np_ptr(sb), _np_ptr(nb), int(elem_offset),
          _ptr(shares), _stream())
    return shares


def ass_reconstruct_wide(shares: torch.Tensor) -> torch.Tensor:
    """int32 [P, l, n] two's-complement limbs -> int32 [l, n] column sum mod 2^(32 l)."""
    lib = N.load()
    shares = shares.contiguous()
    P, L, n = shares.shape
    out = torch.empty((L, n), dtype=torch.int32, device=shares.device)
    _call(lib.fbm_ass_reconstruct_wide, _ptr(shares), int(P), int(L), n, _ptr(out), _stream())
    return out


def ints_to_limbs_tc(values: Sequence[int], n_limbs: int) -> np.ndarray:
    """Python ints -> int32 [n_limbs, n] two's-complement u32 limbs, limb-major."""
    mod = 1 << (32 * n_limbs)
    blob = b"".join((int(v) % mod).to_bytes(4 * n_limbs, "little") for v in values)
    return np.frombuffer(blob, dtype="<u4").reshape(len(values), n_limbs).T.copy().view(np.int32)


def limbs_tc_to_ints(arr: np.ndarray) -> List[int]:
    """int32 [n_limbs, n] two's-complement limbs (limb-major) -> Python ints."""
    L = arr.shape[0]
    rows = np.ascontiguousarray(arr.view(np.uint32).T).astype("<u4")
    top = 1 << (32 * L - 1)
    out = []
    for r in rows:
        w = int.from_bytes(r.tobytes(), "little")
        out.append(w - (top << 1) if w & top else w)
    return out


def reference_share_draws(bls: Sequence[int], draws: int) -> List[List[int]]:
    """The reference's additive-share draws from the global `random`, exactly (`_additive_ss.py:94-96`):
    random.randint(0, 2**bl) for every element (outer) and share (inner); rows [draws][n].  The C module
    runs CPython's MT19937 from random.getstate() and hands the state back with random.setstate(), so the
    stream continues where the reference's would (bit lengths up to 126; past that, or without the
    module, the same calls through `random` itself)."""
    import random

    n = len(bls)
    m = _pyconv()
    if draws <= 0 or n == 0:
        return [[] for _ in range(max(draws, 0))]
    if m is _PyConvFallback or max(bls) > 126:
        cols = [[random.randint(0, 2**bl) for _ in range(draws)] for bl in bls]
        return [[c[j] for c in cols] for j in range(draws)]
    version, state, gauss = random.getstate()
    out = np.empty((draws, n, 2), dtype=np.int64)
    new = m.mt_share_draws(state, np.asarray(bls, dtype=np.uint32).tobytes(), draws, out)
    random.setstate((version, new, gauss))
    return [int128_to_ints(out[j]) for j in range(draws)]


def ints_to_int128(values: Sequence[int]) -> np.ndarray:
    """Python ints in [-2^127, 2^127) -> int64 [n, 2] (lo, hi) two's complement."""
    out = np.empty((len(values), 2), dtype=np.int64)
    u = out.view(np.uint64)
    for i, v in enumerate(values):
        v = int(v)
        if not -(2**127) <= v < 2**127:
            raise ValueError("value outside the int128 range of the device additive-sharing path")
        w = v & (2**128 - 1)
        u[i, 0] = w & (2**64 - 1)
        u[i, 1] = w >> 64
    return out


def int128_to_ints(arr: np.ndarray) -> List[int]:
    u = np.ascontiguousarray(arr).view(np.uint64).reshape(-1, 2)
    out = []
    for lo, hi in u.tolist():
        w = (hi << 64) | lo
        out.append(w - 2**128 if w >> 127 else w)
    return out
