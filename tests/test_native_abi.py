"""CPU-side checks of the drop-in boundary: the C-ABI library builds/loads, exports exactly the
symbols include/fbm_secagg.h declares (the test build: + include/fbm_secagg_test.h), and the
host-side parameter logic matches the reference's Python formulas.  No GPU compute is called here."""

import ctypes
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fbm_secagg.h")
TEST_HEADER = os.path.join(ROOT, "include", "fbm_secagg_test.h")


def declared_symbols(header=HEADER):
    text = open(header).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|uint64_t|const char\*)\s+(fbm_\w+)\s*\(", text, re.M)))


def exported(path):
    """The library's dynamic function exports (nm -D --defined-only, text symbols)."""
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines() if len(ln.split()) == 3 and ln.split()[1] in "TtWi"})


@pytest.fixture(scope="module")
def lib():
    from fedbiomed_amd import _build, _native

    _build.build()
    return _native.load()


def test_header_declares_abi():
    syms = declared_symbols()
    assert "fbm_lom_protect" in syms and "fbm_jl_encrypt" in syms and "fbm_jl_aggregate" in syms
    assert len(syms) >= 10


def test_library_exports_every_declared_symbol(lib):
    from fedbiomed_amd import _native

    for s in declared_symbols():
        assert hasattr(lib, s), f"missing export {s}"
        assert s in _native.SIGNATURES, f"no ctypes signature for {s}"
    assert lib.fbm_abi_version() == _native.ABI_VERSION == 7
    assert set(_native.SIGNATURES) == set(declared_symbols())
    assert set(_native.TEST_SIGNATURES) == set(declared_symbols(TEST_HEADER))


def test_product_library_exports_exactly_its_header(lib):
    """`nm -D` of the shipped library is the set include/fbm_secagg.h documents -- no
    test, A/B or profiling hook, no internal C++ symbol; the test build adds exactly
    include/fbm_secagg_test.h's."""
    from fedbiomed_amd import _native

    prod, test = exported(_native.LIB_PATH), exported(_native.TEST_LIB_PATH)
    assert prod == declared_symbols(), set(prod) ^ set(declared_symbols())
    assert test == sorted(set(declared_symbols()) | set(declared_symbols(TEST_HEADER)))
    assert not any(n.startswith(("fbm_test_", "fbm_prof_")) for n in prod)
    assert not {"fbm_jl_set_engine", "fbm_jl_set_short", "fbm_jl_engine_for"} & set(prod)
    t = _native.load_test()
    assert t is not lib and t.fbm_abi_version() == lib.fbm_abi_version()


def test_test_hooks_route_only_this_thread(lib):
    """_native.test_hooks() sends the calling thread's load() to the test build and no other thread's."""
    import threading

    from fedbiomed_amd import _native

    seen = {}
    with _native.test_hooks():
        assert _native.load() is _native.load_test()
        t = threading.Thread(target=lambda: seen.setdefault("other", _native.load()))
        t.start()
        t.join()
    assert seen["other"] is lib and _native.load() is lib


def test_engine_policy_is_per_thread():
    """the test build's engine / short-path switches are the calling thread's (the
    product library has none); a switch on one thread leaves another thread's policy alone."""
    import threading

    from fedbiomed_amd import _native

    t = _native.load_test()
    prev = t.fbm_jl_set_engine(3)
    try:
        other = {}

        def probe():
            other["engine"] = t.fbm_jl_engine_for(10**7)  # auto here: the one-lane engine
            other["prev_short"] = t.fbm_jl_set_short(0)
            t.fbm_jl_set_short(other["prev_short"])

        th = threading.Thread(target=probe)
        th.start()
        th.join()
        assert other == {"engine": 1, "prev_short": 1}
        assert t.fbm_jl_engine_for(10**7) == 3  # this thread's policy stands
    finally:
        t.fbm_jl_set_engine(prev)


def test_check_stats_lom_guard(lib):
    # host-only helper: error iff max_bits >= 64 - ceil(log2(P))  (_lom.py:133-150)
    def rc(max_bits, nodes):
        st = np.array([max_bits, 0, 0, 0], dtype=np.uint32)
        return lib.fbm_check_stats(ctypes.c_void_p(st.ctypes.data), nodes, None)

    for nodes in (1, 2, 3, 4, 5, 16, 17):
        limit = 64 - math.ceil(math.log2(nodes))
        assert rc(limit - 1, nodes) == 0
        assert rc(limit, nodes) == -4
    st = np.array([0, 1, 0, 0], dtype=np.uint32)  # dequant range flag
    assert lib.fbm_check_stats(ctypes.c_void_p(st.ctypes.data), 0, None) == -3


def test_jl_slot_matches_reference_formula():
    from fedbiomed_amd import _device as D
    from oracle import secagg_oracle as O

    for T in (2**13, 2**55, 10, 2**20 + 3):
        for P in (1, 2, 3, 4, 7, 8, 15, 16, 100):
            assert D.jl_slot(T, P) == O.jl_slot(T, P)
    assert D.jl_slot(None, 8) == (34, 30)
    assert D.jl_slot(None, 4) == (33, 31)


def test_quant_params_semantics():
    from fedbiomed_amd import _device as D

    assert D.quant_params(None, 2**13) == (3.0, 6.0, 8192.0, 8191)
    with pytest.raises(OverflowError):
        D.quant_params(7, 2**64 + 1)
    with pytest.raises(ZeroDivisionError):
        D.dequant_params(3, 1)
    negc, step = D.dequant_params(3, 2**13)
    assert negc == -3.0 and step == 6 / 8191


def test_limb_roundtrip():
    from fedbiomed_amd import _device as D

    rng = np.random.default_rng(0)
    vals = [int.from_bytes(rng.bytes(256), "little") for _ in range(17)] + [0, 1, 2**2048 - 1]
    arr = D.ints_to_limbs(vals)
    assert arr.shape == (len(vals), 64)
    assert D.limbs_to_ints(arr) == vals
    n2 = 12345**2
    assert D.limbs_to_ints(D.ints_to_limbs([-5, 2**2048 + 7], n2)) == [(-5) % n2, (2**2048 + 7) % n2]


def _imported_modules(path):
    """Every module name an Import / ImportFrom node of `path` names (any nesting level:
    module body, functions, try blocks), plus importlib-style string imports."""
    import ast

    tree = ast.parse(open(path).read(), filename=path)
    names = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            names += [a.name for a in node.names]
        elif isinstance(node, ast.ImportFrom):
            mod = node.module or ""
            names += [mod] + [f"{mod}.{a.name}" if mod else a.name for a in node.names]
        elif isinstance(node, ast.Call):  # importlib.import_module("oracle...") / __import__("oracle")
            fn = node.func
            fname = fn.attr if isinstance(fn, ast.Attribute) else getattr(fn, "id", "")
            if fname in ("import_module", "__import__") and node.args and isinstance(node.args[0], ast.Constant):
                names.append(str(node.args[0].value))
    return names


def test_product_path_does_not_import_oracle():
    """The product must never route through the CPU oracle: no module under fedbiomed_amd/
    imports `oracle` (or anything under it), at any nesting level."""
    checked = 0
    for dirpath, _, files in os.walk(os.path.join(ROOT, "fedbiomed_amd")):
        for f in files:
            if f.endswith(".py"):
                path = os.path.join(dirpath, f)
                bad = [m for m in _imported_modules(path) if m == "oracle" or m.startswith("oracle.")
                       or ".oracle" in m or m.endswith("secagg_oracle")]
                assert not bad, (path, bad)
                checked += 1
    assert checked >= 10


def test_oracle_import_guard_catches_regressions(tmp_path):
    """The scan above flags every import form (a guard that cannot fail proves nothing)."""
    for src in ("import oracle", "from oracle import secagg_oracle as O", "import oracle.secagg_oracle",
                "def f():\n    from oracle.secagg_oracle import quantize\n",
                "try:\n    import numpy\nexcept ImportError:\n    import oracle\n",
                "import importlib\nimportlib.import_module('oracle.secagg_oracle')",
                "x = 'docstring mentioning oracle first'\nimport os\nfrom oracle import x"):
        p = tmp_path / "m.py"
        p.write_text(src)
        mods = _imported_modules(str(p))
        assert any(m == "oracle" or m.startswith("oracle.") for m in mods), src
    p = tmp_path / "ok.py"
    p.write_text('"""talks about the oracle"""\nimport os  # oracle in a comment\n')
    assert not any("oracle" in m for m in _imported_modules(str(p)))


def test_device_modinv_on_host():
    """The device modular inverse (Bernstein-Yang divsteps) run through the host test hook
    against Python's pow(x, -1, N): random 1024-bit and small odd moduli, edge inputs,
    non-invertible inputs; batch count within the constant-time bound."""
    import ctypes
    import random

    import numpy as np

    from fedbiomed_amd import _native as N
    from fedbiomed_amd.workload import BIPRIME0

    lib = N.load_test()  # fbm_test_modinv (include/fbm_secagg_test.h)

    def limbs(v):
        return np.frombuffer(int(v).to_bytes(128, "little"), dtype=np.uint32).copy()

    def inv(x, n):
        xa, na, out = limbs(x), limbs(n), np.zeros(32, dtype=np.uint32)
        b = ctypes.c_int(0)
        rc = lib.fbm_test_modinv(xa.ctypes.data, na.ctypes.data, out.ctypes.data, ctypes.byref(b))
        return rc, int.from_bytes(out.tobytes(), "little"), b.value

    rng = random.Random(5)
    moduli = [BIPRIME0, 3, 15, 123457, 2**1024 - 1, (1 << 1023) + 1, rng.getrandbits(1024) | 1 | (1 << 1023)]
    worst = 0
    for n in moduli:
        xs = [1, 2, n - 1, n - 2, (n + 1) // 2] + [rng.randrange(1, n) for _ in range(60)]
        for x in xs:
            x %= n
            rc, got, b = inv(x, n)
            worst = max(worst, b)
            try:
                want = pow(x, -1, n)
            except ValueError:
                assert rc == N.FBM_E_INVERSE, (n, x)
                continue
            assert rc == N.FBM_OK and got == want, (n, x)
    assert inv(0, BIPRIME0)[0] == N.FBM_E_INVERSE
    assert inv(15, 45)[0] == N.FBM_E_INVERSE
    assert worst <= 99


def test_fdh_gcd_on_host():
    """The FDH's one-digest coprimality test (Montgomery reduction of N by the odd part of
    the digest, then a binary gcd) against math.gcd, on the host: random digests, digests
    sharing a factor with N, zero, powers of two, and moduli from 3 to 1024 bits."""
    import random

    from fedbiomed_amd import workload as W

    from fedbiomed_amd import _native

    lib = _native.load_test()  # fbm_test_fdh_gcd (include/fbm_secagg_test.h)
    rng = random.Random(11)
    moduli = [W.BIPRIME0, 3, 9, 15, 3 * 5 * 7 * 11 * 13 * 17 * 19 * 23, (1 << 1024) - 1,
              rng.getrandbits(1024) | 1, rng.getrandbits(300) | 1]
    p, q = 1000003, 998244353
    moduli.append(p * q)
    for N in moduli:
        n32 = np.frombuffer(N.to_bytes(128, "little"), dtype=np.uint32).copy()
        cases = [0, 1, 2, 1 << 255, (1 << 256) - 1, N % (1 << 256)]
        cases += [rng.getrandbits(256) for _ in range(40)]
        for f in (3, 5, 7, p, q):
            if N % f == 0:
                cases += [(rng.getrandbits(200) * f) % (1 << 256) for _ in range(5)]
        for r in cases:
            r8 = np.frombuffer(r.to_bytes(32, "little"), dtype=np.uint32).copy()
            err = ctypes.c_uint32(0)
            got = lib.fbm_test_fdh_gcd(r8.ctypes.data, n32.ctypes.data, ctypes.byref(err))
            assert got == int(math.gcd(r, N) == 1), (N, r)
            assert err.value == 0


def _stub_lib(tmp_path, abi):
    """A library with fbm_abi_version() only -- every other entry point missing."""
    src = tmp_path / "stub.c"
    src.write_text(f"int fbm_abi_version(void) {{ return {abi}; }}\n")
    so = tmp_path / f"libstub{abi}.so"
    import subprocess
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    return str(so)


def _load_in_child(env_extra):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (f"import sys; sys.path.insert(0, {root!r})\n"
            "from fedbiomed_amd import _native as N\n"
            "try:\n    N.load(); print('LOADED', N.loaded_abi)\n"
            "except N.NativeUnavailable as e:\n    print('REFUSED', e)\n")
    env = dict(os.environ)
    env.pop("FBM_AB_VARIANT", None)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


def test_lib_path_override_alone_is_strict(tmp_path):
    """FBM_LIB_PATH alone: the override is loaded under the shipped checks -- a library missing
    entry points is NativeUnavailable at load(), not an AttributeError at first use."""
    from fedbiomed_amd import _native as N
    out = _load_in_child({"FBM_LIB_PATH": _stub_lib(tmp_path, N.ABI_VERSION)})
    assert out.startswith("REFUSED") and "lacks" in out, out
    out = _load_in_child({"FBM_LIB_PATH": _stub_lib(tmp_path, N.ABI_VERSION - 1)})
    assert out.startswith("REFUSED"), out


def test_lib_path_override_relaxed_only_for_ab_variants(tmp_path):
    from fedbiomed_amd import _native as N
    out = _load_in_child({"FBM_LIB_PATH": _stub_lib(tmp_path, N.ABI_VERSION - 1), "FBM_AB_VARIANT": "1"})
    assert out == f"LOADED {N.ABI_VERSION - 1}", out
    out = _load_in_child({"FBM_LIB_PATH": _stub_lib(tmp_path, N.ABI_VERSION - 2), "FBM_AB_VARIANT": "1"})
    assert out.startswith("REFUSED") and "ABI version mismatch" in out, out


def test_abi2_variant_refuses_wide_rounds():
    from fedbiomed_amd import _device as D, _native as N
    from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError
    saved = N.loaded_abi
    try:
        N.loaded_abi = 2
        assert D._check_round(2 ** 512 - 1)[15] == 0xFFFFFFFF
        with pytest.raises(FedbiomedSecaggCrypterError):
            D._check_round(2 ** 512)
        N.loaded_abi = 3
        assert D._check_round(2 ** 512)[16] == 1
    finally:
        N.loaded_abi = saved


def test_lib_path_override_serves_both_builds():
    """FBM_LIB_PATH (an A/B variant, built with the test build's exports) is both load() and load_test(): one
    CDLL, and the test header's signatures set on it even when load() opened it first."""
    import subprocess
    import sys

    from fedbiomed_amd import _build, _native as N

    _build.build()
    code = (f"import sys; sys.path.insert(0, {ROOT!r})\n"
            "import ctypes\n"
            "from fedbiomed_amd import _native as N\n"
            "a = N.load(); t = N.load_test()\n"
            "assert t is a is N.load()\n"
            "assert t.fbm_jl_engine_for.argtypes == [ctypes.c_uint64]\n"
            "assert t.fbm_jl_engine_for(333334) == 1\n"
            "print('OK')\n")
    env = dict(os.environ, FBM_LIB_PATH=N.TEST_LIB_PATH)
    env.pop("FBM_AB_VARIANT", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stderr
