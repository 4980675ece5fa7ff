"""List-API host conversions (csrc/fbm_pyconv.c) against Python's own conversions.

The reference crypters take and return Python lists (`_secagg_crypter.py:45-230`); the C
loops must give exactly what `array('d', ...)`, `int.to_bytes` / `int.from_bytes` and
`np.array(..., dtype=uint64)` give, and hand every value they cannot convert back to the
Python path (reduction mod N^2, numpy's errors).  CPU only.
"""

import array
import os
import random

import numpy as np
import pytest

from fedbiomed_amd import _device as D
from fedbiomed_amd.secagg._secagg_crypter import _check_float_list
from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError


class F(float):
    pass


def test_floats_match_array_d():
    rng = random.Random(3)
    vals = [rng.uniform(-1e6, 1e6) for _ in range(5000)] + [0.0, -0.0, float("inf"), float("-inf"),
                                                           float("nan"), 5e-324, 1.7976931348623157e308, F(2.5)]
    got = _check_float_list(vals).numpy()
    ref = np.frombuffer(array.array("d", vals), dtype=np.float64)
    assert got.tobytes() == ref.tobytes()  # bit patterns, NaN and -0.0 included
    assert _check_float_list([]).numel() == 0


@pytest.mark.parametrize("bad", [[1.0, 2, 3.0], [1.0, "x"], [None], [np.float32(1.0)], [True]])
def test_float_check_rejects_what_isinstance_rejects(bad):
    assert not all(isinstance(v, float) for v in bad)
    with pytest.raises(FedbiomedSecaggCrypterError):
        _check_float_list(bad)


def test_float_subclasses_pass():
    vals = [np.float64(0.25), F(1.5), 3.0]
    assert all(isinstance(v, float) for v in vals)
    assert _check_float_list(vals).tolist() == [0.25, 1.5, 3.0]


def test_ints_to_limbs_matches_to_bytes():
    rng = random.Random(5)
    vals = [0, 1, 2**30 - 1, 2**30, 2**32, 2**60, 2**64 - 1, 2**2047, 2**2048 - 1, True]
    vals += [rng.getrandbits(rng.randint(1, 2048)) for _ in range(3000)]
    got = D.ints_to_limbs(vals)
    ref = np.frombuffer(b"".join(int(v).to_bytes(256, "little") for v in vals), dtype=np.uint32).reshape(-1, 64)
    assert np.array_equal(got, ref)
    assert D.limbs_to_ints(got) == [int(v) for v in vals]


def test_ints_to_limbs_out_of_range_values_reduced():
    n2 = (2**1023 + 1155) ** 2
    vals = [7, -5, 2**2048, 2**2100 + 9, np.int64(11), 3, -(2**3000)]
    got = D.limbs_to_ints(D.ints_to_limbs(vals, n2))
    assert got == [7, (-5) % n2, 2**2048 % n2, (2**2100 + 9) % n2, 11, 3, (-(2**3000)) % n2]
    with pytest.raises(OverflowError):
        D.ints_to_limbs([1, -1])  # no modulus to reduce by


def test_ints_to_limbs_into_row_views():
    rng = random.Random(9)
    rows = [[rng.getrandbits(2048) for _ in range(17)] for _ in range(3)]
    out = np.zeros((3, 17, 64), dtype=np.uint32)
    for u, r in enumerate(rows):
        D.ints_to_limbs(r, None, out=out[u])
    assert [D.limbs_to_ints(out[u]) for u in range(3)] == rows


def test_u64_rows_match_numpy_and_its_errors():
    rng = random.Random(11)
    rows = [[rng.getrandbits(64) for _ in range(1000)] for _ in range(4)]
    rows[1][3] = 2**64 - 1
    m = D._pyconv()
    buf = np.empty((4, 1000), dtype=np.int64)
    assert all(m.ints_to_bytes(r, 8, buf[u]) < 0 for u, r in enumerate(rows))
    assert np.array_equal(buf.view(np.uint64), np.array(rows, dtype=np.uint64))
    for bad in (-1, 2**64, 1.5, "7"):
        assert m.ints_to_bytes([1, 2, bad], 8, np.empty(3, np.int64)) == 2


def test_buffer_size_checked():
    m = D._pyconv()
    with pytest.raises(ValueError):
        m.ints_to_bytes([1, 2], 8, np.empty(3, np.int64))
    with pytest.raises(ValueError):
        m.floats_to_f64([1.0], np.empty(2, np.float64))
    with pytest.raises(ValueError):
        m.bytes_to_ints(b"\0" * 10, 4)


@pytest.mark.parametrize("threads", ["1", "3", "8"])
def test_threaded_ints_to_bytes_first_bad_index(monkeypatch, threads):
    """Ciphertext-sized lists (>= 1 MB of output) convert on several threads with the GIL
    released; the answer (bytes and first bad index) must not depend on the thread count."""
    monkeypatch.setenv("FBM_CONV_THREADS", threads)
    m = D._pyconv()
    rng = random.Random(12)
    vals = [rng.getrandbits(2048) for _ in range(6000)]
    vals[:6] = [0, 1, 2**30 - 1, 2**30, 2**32, 2**2048 - 1]
    out = np.empty((len(vals), 64), dtype=np.uint32)
    assert m.ints_to_bytes(vals, 256, out) == -1
    assert out.tobytes() == b"".join(v.to_bytes(256, "little") for v in vals)
    for bad_at, bad in ((5999, -3), (4500, 2**2048), (2100, 1.0), (3, "x")):
        v2 = list(vals)
        v2[bad_at] = bad
        v2[5998] = -1  # a later bad item in another range: the first one is reported
        assert m.ints_to_bytes(v2, 256, out) == min(bad_at, 5998)
    # and back: 6000 x 256 B is past the threaded size, so the digits are written on host threads
    assert m.ints_to_bytes(vals, 256, out) == -1
    back = m.bytes_to_ints(out, 256)
    assert back == vals and all(type(v) is int for v in back)
    assert all(v is w for v, w in zip(back[:2], range(2)))  # the small-int cache, never written by the fill


def test_bytes_to_ints_word_path_edges():
    m = D._pyconv()
    vals = [0, 1, 255, 256, 2**30 - 1, 2**30, 2**31, 2**32 - 1, 2**32, 2**60, 2**2047, 2**2048 - 1]
    vals += [random.Random(13).getrandbits(b) for b in range(1, 2049, 37)]
    blob = np.frombuffer(b"".join(v.to_bytes(256, "little") for v in vals), dtype=np.uint32)
    got = m.bytes_to_ints(blob, 256)
    assert got == vals and all(type(v) is int for v in got)
    assert m.bytes_to_ints(b"\x05\0\0", 3) == [5]  # byte path (width not a word multiple)


def test_deferred_checks_are_per_thread():
    """A status word deferred inside one thread's `deferred_checks` (the list aggregate issues
    its decryption factor that way) never lands in another thread's context."""
    import threading

    seen = {}
    with D.deferred_checks():
        D.deferred_checks._stack()[-1].append(("main", 0))

        def other():
            seen["other"] = list(D.deferred_checks._stack())

        t = threading.Thread(target=other)
        t.start()
        t.join()
        assert len(D.deferred_checks._stack()[-1]) == 1
        D.deferred_checks._stack()[-1].clear()  # nothing to check at exit (no device here)
    assert seen["other"] == [] and D.deferred_checks._stack() == []


# ---- the three implementations of the conversion contract ---------------------------------
# the in-tree C module, the same source built with the version-portable byte-API path
# (-DFBM_DIGITS_FAST=0: what CPython >= 3.12 compiles), and the pure-Python fallback the list
# API uses when the module is not built for the running interpreter.
@pytest.fixture(scope="module", params=["c", "portable_c", "python"])
def conv(request, tmp_path_factory):
    if request.param == "python":
        return D._PyConvFallback
    if request.param == "c":
        m = D._pyconv()
        if m is D._PyConvFallback:
            pytest.skip("C conversion module not built")
        return m
    import importlib.util
    import shutil
    import subprocess
    import sysconfig

    from fedbiomed_amd import _build

    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    out = tmp_path_factory.mktemp("pyconv") / ("_fbm_pyconv" + sysconfig.get_config_var("EXT_SUFFIX"))
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-Wall", "-Werror", "-pthread", "-DFBM_DIGITS_FAST=0",
                    "-I" + sysconfig.get_paths()["include"], _build.PYCONV_SRC, "-o", str(out)], check=True)
    spec = importlib.util.spec_from_file_location("_fbm_pyconv", str(out))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_conv_contract_ints(conv):
    rng = random.Random(21)
    vals = [0, 1, 2**30 - 1, 2**30, 2**32, 2**2047, 2**2048 - 1] + [rng.getrandbits(2040) for _ in range(500)]
    out = np.empty((len(vals), 64), dtype=np.uint32)
    assert conv.ints_to_bytes(vals, 256, out) == -1
    assert out.tobytes() == b"".join(v.to_bytes(256, "little") for v in vals)
    assert conv.bytes_to_ints(out, 256) == vals
    for bad in (-1, 2**2048, 1.0, "x"):
        assert conv.ints_to_bytes([5, 6, bad, 7], 256, np.empty((4, 64), np.uint32)) == 2
    u = np.empty(3, np.int64)
    assert conv.ints_to_bytes([1, 2**64 - 1, 0], 8, u) == -1 and u.view(np.uint64).tolist() == [1, 2**64 - 1, 0]
    with pytest.raises(ValueError):
        conv.ints_to_bytes([1, 2], 8, np.empty(3, np.int64))


def test_conv_contract_floats(conv):
    vals = [0.5, -0.0, float("nan"), float("inf"), F(2.5), np.float64(3.25)]
    out = np.empty(len(vals), np.float64)
    assert conv.floats_to_f64(vals, out) == -1
    assert out.tobytes() == np.frombuffer(array.array("d", vals), dtype=np.float64).tobytes()
    assert conv.floats_to_f64([1.0, 2, 3.0], np.empty(3, np.float64)) == 1
    with pytest.raises(ValueError):
        conv.floats_to_f64([1.0], np.empty(2, np.float64))


def test_conv_contract_float_list(conv):
    vals = np.array([0.5, -0.0, float("nan"), float("inf"), 1e-310, -3.75], dtype=np.float64)
    lst = conv.none_list(9)
    assert lst == [None] * 9
    conv.f64_into_list(lst, 2, vals)
    conv.f64_into_list(lst, 8, vals[:1])
    assert lst[:2] == [None, None] and lst[8] == 0.5 and all(type(v) is float for v in lst[2:])
    assert np.array(lst[2:8]).tobytes() == vals.tobytes()
    conv.f64_into_list(lst, 0, vals[:0])
    with pytest.raises(ValueError):
        conv.f64_into_list(lst, 4, vals)  # past the end
    conv.f64_into_list(lst, 1, vals[4:6])  # a filled slot is written again
    assert lst[1] == 1e-310 and lst[2] == -3.75
    lst[3] = "x"
    with pytest.raises(ValueError):
        conv.f64_into_list(lst, 3, vals[:1])  # neither None nor a float
    with pytest.raises(ValueError):
        conv.none_list(-1)
    assert conv.none_list(0) == []


def test_conv_contract_ints_to_bytes_held(conv):
    """The aggregate's per-stripe conversion: items [lo, hi) of every party's list -> out [P, hi - lo, n] on
    host threads in one GIL-held call (no pins); -1 or the first bad flat index u (hi - lo) + i."""
    rng = random.Random(26)
    lists = [[rng.getrandbits(2048) for _ in range(3000)] for _ in range(3)]
    lo, hi = 300, 2700
    out = np.empty((3, hi - lo, 64), np.uint32)
    ref = np.empty_like(out)
    for u in range(3):
        assert conv.ints_to_bytes(lists[u][lo:hi], 256, ref[u]) == -1
    assert conv.ints_to_bytes_held(lists, lo, hi, 256, out) == -1
    assert out.tobytes() == ref.tobytes()
    bad = [list(v) for v in lists]
    bad[2][lo + 9] = -1
    bad[1][lo + 3] = "x"
    assert conv.ints_to_bytes_held(bad, lo, hi, 256, out) == (hi - lo) + 3
    bad[1][lo + 3] = 5
    bad[0][hi] = "outside the range"  # not converted, not reported
    assert conv.ints_to_bytes_held(bad, lo, hi, 256, out) == 2 * (hi - lo) + 9
    assert conv.ints_to_bytes_held(lists, 5, 5, 256, np.empty((3, 0, 64), np.uint32)) == -1
    for args in ((lists, 0, 3001, 256, np.empty((3, 3001, 64), np.uint32)),  # past a list's end
                 (lists, 0, 10, 256, np.empty((3, 11, 64), np.uint32)),  # buffer size
                 (lists, 0, 10, 6, np.empty((3, 10, 6), np.uint8)),  # width not a word multiple
                 ([lists[0], (1, 2)], 0, 1, 256, np.empty((2, 1, 64), np.uint32))):
        with pytest.raises(ValueError):
            conv.ints_to_bytes_held(*args)


def test_convert_stripe_reduces_out_of_range():
    n2 = (2**1023 + 1155) ** 2
    rng = random.Random(27)
    lists = [[rng.getrandbits(2040) for _ in range(50)] for _ in range(3)]
    lists[1][12] = -7
    lists[2][30] = 2**2050 + 3
    out = np.empty((3, 30, 64), np.uint32)
    D.convert_stripe(lists, 5, 35, n2, out)
    assert [D.limbs_to_ints(out[u]) for u in range(3)] == [[v % n2 for v in lst[5:35]] for lst in lists]


def test_float_pool_filled_in_place():
    """prepare_aggregate's output list made ahead: its floats' values are written in place (the same objects)
    while only the list holds them; a float something else also holds is replaced, never changed."""
    m = D._pyconv()
    pool = m.float_pool(6)
    assert pool == [0.0] * 6 and len({id(v) for v in pool}) == 6
    ids = [id(v) for v in pool]
    held = pool[3]  # a second holder
    m.f64_into_list(pool, 1, np.array([1.5, -2.25, 3.0, float("nan")]))
    assert pool[1:3] == [1.5, -2.25] and [id(v) for v in pool[1:3]] == ids[1:3]  # in place
    assert held == 0.0 and pool[3] == 3.0 and id(pool[3]) != ids[3]  # replaced, the held one unchanged
    assert pool[4] != pool[4] and pool[0] == 0.0 and pool[5] == 0.0
    m.f64_into_list(pool, 0, np.array([7.0, 8.0]))
    assert pool[:2] == [7.0, 8.0] and id(pool[0]) == ids[0]
    with pytest.raises(ValueError):
        m.f64_into_list(["x", 1.0], 0, np.array([1.0]))  # neither None nor a float
    with pytest.raises(ValueError):
        m.float_pool(-1)


@pytest.mark.parametrize("threads", ["1", "7"])
def test_float_pool_filled_on_threads(monkeypatch, threads):
    """Past the threaded size (65 536 slots) the in-place writes run on host threads: the pool's own floats
    written in place, None slots and floats held elsewhere replaced on the calling thread, a bad slot
    anywhere refused before any write."""
    monkeypatch.setenv("FBM_CONV_THREADS", threads)
    m = D._pyconv()
    n = 200_000
    vals = np.random.default_rng(3).standard_normal(n)
    pool = m.float_pool(n)
    ids = [id(v) for v in pool[:1000]]
    pool[5] = None
    held = pool[150_000]
    m.f64_into_list(pool, 0, vals)
    assert np.array(pool).tobytes() == vals.tobytes() and all(type(v) is float for v in pool)
    assert [id(v) for v in pool[:5]] == ids[:5] and held == 0.0 and id(pool[150_000]) != id(held)
    bad = m.float_pool(n)
    bad[123_456] = 1
    with pytest.raises(ValueError):
        m.f64_into_list(bad, 0, vals)
    assert bad[0] == 0.0 and bad[199_999] == 0.0  # nothing written


def test_default_threads_follow_the_cpu_share(monkeypatch):
    """The threaded loops default to the process's CPU share (affinity capped by a cgroup quota), at
    most 16; FBM_CONV_THREADS still overrides it per call."""
    avail = len(os.sched_getaffinity(0))
    monkeypatch.setattr(D, "cgroup_cpu_quota", lambda: 2.5)
    assert D.host_cpu_share() == min(avail, 2)
    monkeypatch.setattr(D, "cgroup_cpu_quota", lambda: None)
    assert D.host_cpu_share() == avail
    m = D._pyconv()
    if m is D._PyConvFallback:
        pytest.skip("C conversion module not built")
    old = m.set_conv_threads(3)
    try:
        assert old == min(16, D.host_cpu_share())
        assert m.set_conv_threads(0) == 3 and m.set_conv_threads(1000) == 1 and m.set_conv_threads(old) == 64
    finally:
        m.set_conv_threads(old)


def test_int_pool_filled_in_place():
    """prepare_encrypt's output list: ints made ahead (value 0), their values written in place later from
    limb rows -- the same ints int.from_bytes makes (normalised: comparisons, hashing and arithmetic agree),
    on host threads past the threaded size; a pool item held elsewhere, a foreign item or a buffer of
    another size is refused before anything is written."""
    m = D._pyconv()
    if m is D._PyConvFallback:
        pytest.skip("C conversion module not built")
    rng = random.Random(31)
    vals = [0, 1, 255, 2**30 - 1, 2**30, 2**32, 2**2047, 2**2048 - 1] + [rng.getrandbits(rng.randint(1, 2048))
                                                                           for _ in range(6000)]
    pool = D.int_pool(len(vals))
    assert len(pool) == len(vals) and all(type(v) is int and v == 0 for v in pool)
    rows = np.frombuffer(b"".join(v.to_bytes(256, "little") for v in vals), np.uint32).reshape(-1, 64)
    assert D.limbs_into_pool(pool, rows) is pool
    assert pool == vals and all(type(v) is int for v in pool)
    assert [hash(v) for v in pool[:50]] == [hash(v) for v in vals[:50]]
    assert sum(pool) == sum(vals) and pool[8] + 1 == vals[8] + 1 and str(pool[7]) == str(vals[7])
    pool2 = D.int_pool(3)
    held = pool2[1]
    with pytest.raises(ValueError):  # refcount 2: someone else holds it
        m.words_into_pool(pool2, rows[:3].tobytes(), 256)
    assert pool2 == [0, 0, 0] and held == 0
    got = D.limbs_into_pool(pool2, rows[:3])  # the device layer then makes a fresh list
    assert got == vals[:3] and got is not pool2 and pool2 == [0, 0, 0] and held == 0
    u64 = np.array([0, 1, 2**64 - 1], np.uint64)
    assert D.u64_into_pool(pool2, u64) == [0, 1, 2**64 - 1] and held == 0
    del held
    with pytest.raises(ValueError):
        m.words_into_pool([0, 5, 2**100], rows[:3].tobytes(), 256)  # not a pool
    with pytest.raises(ValueError):
        m.words_into_pool(D.int_pool(2), rows[:3].tobytes(), 256)  # size
    # by slices (the striped encrypt): rows [3, 7) at offset 3, the rest left at 0; past the end refused
    pool3 = D.int_pool(10)
    assert D.limbs_into_pool(pool3, rows[8:12], 3, strict=True) is pool3
    assert pool3 == [0, 0, 0] + vals[8:12] + [0, 0, 0]
    with pytest.raises(ValueError):
        D.limbs_into_pool(pool3, rows[:4], 7, strict=True)
    with pytest.raises(ValueError):
        m.words_into_pool(pool3, rows[:1].tobytes(), 256, -1)


def test_int_pool_absent_from_the_portable_build(tmp_path):
    import importlib.util
    import shutil
    import subprocess
    import sysconfig

    from fedbiomed_amd import _build

    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    out = tmp_path / ("_fbm_pyconv" + sysconfig.get_config_var("EXT_SUFFIX"))
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-Wall", "-Werror", "-pthread", "-DFBM_DIGITS_FAST=0",
                    "-I" + sysconfig.get_paths()["include"], _build.PYCONV_SRC, "-o", str(out)], check=True)
    spec = importlib.util.spec_from_file_location("_fbm_pyconv", str(out))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.int_pool(4, 256) is None
    with pytest.raises(ValueError):
        mod.words_into_pool([0], bytes(256), 256)


@pytest.mark.parametrize("threads", ["1", "5"])
def test_all_ints_lists(conv, monkeypatch, threads):
    """The researcher's type check of every party's list in one pass: -1, or the first list with a
    non-int (bool and int subclasses are ints, as isinstance says); empty lists anywhere."""
    monkeypatch.setenv("FBM_CONV_THREADS", threads)
    rng = random.Random(41)
    lists = [[rng.getrandbits(64) for _ in range(30_000)] for _ in range(4)] + [[]] + [[1, True, 2**3000]]
    assert conv.all_ints_lists(lists) == -1
    assert conv.all_ints_lists([]) == -1 and conv.all_ints_lists([[], []]) == -1
    for u, i, bad in ((0, 0, 1.0), (2, 29_999, "x"), (3, 15_000, None), (5, 2, 2.5)):
        l2 = [list(r) for r in lists]
        l2[u][i] = bad
        assert conv.all_ints_lists(l2) == u
        if u < 5:  # a later bad list never hides an earlier one
            l2[5][0] = 0.5
            assert conv.all_ints_lists(l2) == u
    with pytest.raises(TypeError):
        conv.all_ints_lists([[1], (2,)])


def test_reference_share_draws_are_python_random():
    """AdditiveSecret.split(reference_rng=True)'s draws: CPython's MT19937 run in C from random.getstate() --
    the same values random.randint(0, 2**bl) gives, element-major (the reference's loop order), for bit
    lengths around every 32-bit word boundary, and `random` left in the same state; past 126 bits the
    module hands over to `random` itself."""
    import random as R

    bls = [0, 1, 2, 5, 31, 32, 33, 63, 64, 65, 95, 96, 97, 126, 13, 13, 13]
    for seed in (99, 12345):
        R.seed(seed)
        ref = [[R.randint(0, 2**bl) for _ in range(4)] for bl in bls]
        ref_state = R.getstate()
        R.seed(seed)
        got = D.reference_share_draws(bls, 4)
        assert got == [[c[j] for c in ref] for j in range(4)]
        assert R.getstate() == ref_state
    R.seed(5)
    a = D.reference_share_draws([127, 3], 2)  # past 126 bits: through `random`
    R.seed(5)
    ref = [[R.randint(0, 2**127) for _ in range(2)], [R.randint(0, 2**3) for _ in range(2)]]
    assert a == [[ref[0][j], ref[1][j]] for j in range(2)]
    assert D.reference_share_draws([], 3) == [[], [], []] and D.reference_share_draws([4], 0) == []


def _build_pyconv(tmp_path, *defines):
    import importlib.util
    import shutil
    import subprocess
    import sysconfig

    from fedbiomed_amd import _build

    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    out = tmp_path / ("_fbm_pyconv" + sysconfig.get_config_var("EXT_SUFFIX"))
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-Wall", "-Werror", "-pthread", *defines,
                    "-I" + sysconfig.get_paths()["include"], _build.PYCONV_SRC, "-o", str(out)], check=True)
    spec = importlib.util.spec_from_file_location("_fbm_pyconv", str(out))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_inplace_writes_only_on_cpython_310_311(tmp_path, monkeypatch):
    """writes into objects made ahead (an int_pool int's digits, a float_pool float's value)
    happen only on CPython 3.10 / 3.11.  The Python gate refuses every other version whatever the build; a
    build without them (-DFBM_INPLACE=0, what another interpreter compiles) makes no int pools, and its
    f64_into_list replaces a pool's floats by new ones instead of writing them; the unprepared list calls
    take none of it unless INPLACE_UNPREPARED."""
    import sys as _sys

    assert D.inplace_allowed((3, 10, 12)) and D.inplace_allowed((3, 11, 0))
    for v in ((3, 9, 18), (3, 12, 0), (3, 13, 1), (4, 0, 0)):
        assert not D.inplace_allowed(v), v
    assert D.inplace_allowed() == (_sys.version_info[:2] in ((3, 10), (3, 11)))
    m = D._pyconv()
    if m is not D._PyConvFallback:
        assert tuple(m.build_flags()) == ((1, 1) if D.inplace_allowed() else (0, 0))
    # an interpreter outside the gate: no pools, whatever the module
    monkeypatch.setattr(D, "inplace_allowed", lambda version=None: False)
    assert D.int_pool(4) is None and D.int_pool(4, 8, prepared=True) is None and not D.inplace(True)
    monkeypatch.undo()
    assert D.int_pool(4, prepared=False) is None  # the unprepared encrypt: INPLACE_UNPREPARED["encrypt"] off
    assert D.inplace(False, "aggregate") == D.inplace(True)  # the unprepared aggregate keeps its (11 % gain)
    # the build without in-place writes
    mod = _build_pyconv(tmp_path, "-DFBM_INPLACE=0")
    assert tuple(mod.build_flags()) == (0, 1 if D.inplace_allowed() else 0)
    assert mod.int_pool(4, 256) is None
    with pytest.raises(ValueError):
        mod.words_into_pool([0], bytes(256), 256)
    for n in (5, 100_000):  # one thread, and the threaded check / fill passes
        pool = mod.float_pool(n)
        ids = [id(v) for v in pool[:5]]
        keep = pool[3]  # a float held elsewhere too: never written, replaced
        vals = np.arange(n, dtype=np.float64) * 0.5
        mod.f64_into_list(pool, 0, vals)
        assert pool == vals.tolist() and keep == 0.0
        assert all(id(v) != i for v, i in zip(pool[:5], ids) if v != 0.0)  # new objects, not overwritten
