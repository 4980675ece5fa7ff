"""Even (and other non-Montgomery) biprimes: the generic engine (fedbiomed_amd/csrc/fbm_gen.hip).

The reference computes with any N (gmpy2 powmod / invert, Python ints: _jls.py:37-73, 473-562),
and two of its caller tests pass even biprimes -- tests/test_node_secagg.py:207-221 (N = 1156)
and tests/test_secure_aggregation.py:193-233 (N = 1234).  Pinned here by the reference's own
outputs on exactly those inputs and on a seeded sweep of even moduli of 2..1024 bits
(tests/golden/even.json, tools/gen_golden.py gen_even), on the CPU (the engine's per-ciphertext
arithmetic through the host test hooks fbm_test_gen_exp / fbm_test_gen_combine, against the
oracle and the fixtures) and on the GPU (every JL entry point through the C-ABI: the crypters, the
object API, the generic engine against the Montgomery engines on odd moduli)."""

import ctypes
import logging
import math
import random

import numpy as np
import pytest

from fedbiomed_amd import workload as W
from oracle import secagg_oracle as O
from tests.golden_util import F, I


def _limbs(v: int, n: int) -> np.ndarray:
    return np.frombuffer(int(v).to_bytes(4 * n, "little"), dtype=np.uint32).copy()


def _int(a: np.ndarray) -> int:
    return int.from_bytes(np.ascontiguousarray(a, dtype=np.uint32).tobytes(), "little")


def _bits(xs):
    return np.asarray(xs, dtype=np.float64).view(np.uint64).tolist()


def _run(outcome, fn):
    if "error" in outcome:
        with pytest.raises(Exception) as ei:
            fn()
        assert type(ei.value).__name__ == outcome["error"]
        assert str(ei.value) == outcome["msg"]
        return None
    return fn()


class _Host:
    """The generic engine's per-ciphertext work run on the host (include/fbm_secagg_test.h hooks)."""

    def __init__(self):
        from fedbiomed_amd import _native as N

        self.lib = N.load_test()
        self.N = N

    def exp(self, h: int, key: int, n: int, pt=None, negative=False) -> int:
        out = np.zeros(64, np.uint32)
        err = ctypes.c_uint32(0)
        bufs = [_limbs(h, 64), None if pt is None else _limbs(pt, 32), _limbs(n, 32), _limbs(abs(key), 64)]
        p = [None if b is None else ctypes.c_void_p(b.ctypes.data) for b in bufs]
        rc = self.lib.fbm_test_gen_exp(p[0], p[1], 1 if negative else 0, p[2], p[3], 1 if key < 0 else 0,
                                       ctypes.c_void_p(out.ctypes.data), ctypes.byref(err))
        assert rc == 0, self.N.last_error()
        assert err.value == 0
        return _int(out)

    def combine(self, cts, n: int, factor=None, decrypt=False) -> int:
        out = np.zeros(64, np.uint32)
        err = ctypes.c_uint32(0)
        rows = np.concatenate([_limbs(c, 64) for c in cts])
        fb = None if factor is None else _limbs(factor, 64)
        nb = _limbs(n, 32)
        rc = self.lib.fbm_test_gen_combine(ctypes.c_void_p(rows.ctypes.data), len(cts),
                                           None if fb is None else ctypes.c_void_p(fb.ctypes.data),
                                           ctypes.c_void_p(nb.ctypes.data), 1 if decrypt else 0,
                                           ctypes.c_void_p(out.ctypes.data), ctypes.byref(err))
        assert rc == 0, self.N.last_error()
        assert err.value == 0
        return _int(out[:32] if decrypt else out)


@pytest.fixture(scope="module")
def host():
    return _Host()


# ------------------------------------------------------------------ CPU: the arithmetic
def _moduli(rng):
    out = [2, 4, 6, 8, 1156, 1234, 2**32, 2**33, 2**64, 2**64 + 2, 3 * 2**40, 2**1023, (2**1024 - 1) - 1]
    for b in (3, 9, 17, 31, 32, 33, 63, 64, 65, 96, 127, 255, 256, 257, 511, 512, 513, 700, 1000, 1023, 1024):
        out.append((rng.getrandbits(b) | (1 << (b - 1))) & ~1)
        out.append(rng.getrandbits(b) | (1 << (b - 1)) | 1)  # odd moduli take the same engine on request
    return [m for m in out if m >= 2]


def test_generic_powmod_host_vs_oracle(host):
    """h^key mod N^2 (key of either sign: gmpy2's powmod inverts first) times (N pt + 1) mod N^2,
    every size class of even and odd N, keys of 0..2040 bits, h of 8..2048 bits (FDH widths)."""
    rng = random.Random(77)
    for n in _moduli(rng):
        m = n * n
        for _ in range(3):
            while True:
                h = rng.getrandbits(rng.choice([8, 256, 1024, 1792, 2048]))
                if math.gcd(h, m) == 1:
                    break
            key = rng.getrandbits(rng.choice([0, 1, 2, 33, 700, 2040])) * rng.choice([1, -1])
            want = O.powmod(h, key, m)
            assert host.exp(h, key, n) == want, (n, key)
            pt = rng.getrandbits(rng.choice([1, 30, 1024]))
            neg = rng.random() < 0.3
            enc = ((n * (-pt if neg else pt) + 1) % m) * want % m
            assert host.exp(h, key, n, pt=pt, negative=neg) == enc, (n, key, pt, neg)


def test_generic_combine_host_vs_oracle(host):
    """prod_u c_u (* factor) mod N^2 of operands of any size below 2^2048, and the decryption
    ((v - 1) // N) mod N with Python's floor division (v = 0 -> N - 1)."""
    rng = random.Random(78)
    for n in _moduli(rng):
        m = n * n
        for P in (1, 2, 5):
            cts = [rng.getrandbits(rng.choice([1, 64, 2048])) for _ in range(P)]
            f = rng.getrandbits(2048) % m
            v = 1
            for c in cts:
                v = v * c % m
            assert host.combine(cts, n) == v
            vf = v * f % m
            assert host.combine(cts, n, factor=f, decrypt=True) == ((vf - 1) // n) % n
        assert host.combine([0], n, decrypt=True) == n - 1  # a zero product
        assert host.combine([m, 5], n, decrypt=True) == n - 1


def test_node_round_fixture_host(host, golden):
    """tests/test_node_secagg.py:207-221's encrypt (N = 1156) recomputed from the oracle's pack and
    FDH through the generic engine's arithmetic: the reference's ciphertext."""
    c = golden["even"]["node_round"]
    n = c["biprime"]
    es, cr = O.jl_slot(None, c["num_nodes"])
    q = O.quantize(np.array([F(v) for v in c["params"]]), c["clip"])
    pts = O.ves_encode([int(v) * c["weight"] for v in q], es, cr)
    got = [host.exp(O.fdh((k << 512) | c["round"], n * n), c["key"], n, pt=pt) for k, pt in enumerate(pts)]
    assert got == [I(v) for v in c["enc"]["ok"]] == [946993]


def test_even_fixture_object_api_host(host, golden):
    """UserKey.encrypt / sums / ServerKey.decrypt of the fixture's even moduli through the host hooks."""
    for c in golden["even"]["object"]:
        n, tau = I(c["n"]), c["tau"]
        m = n * n
        for key, row in zip(c["keys"], c["ct"]):
            for k, (pt, ct) in enumerate(zip(c["pt"], row)):
                pt = I(pt)  # the object API hands the device pt mod N outside [0, 2^1024)
                h = O.fdh((k << 512) | tau, m)
                got = host.exp(h, I(key), n, pt=pt if 0 <= pt < 2**1024 else pt % n)
                assert got == I(ct), (c["n"], key, pt)
        for k, s in enumerate(c["sum"]):
            assert host.combine([I(r[k]) for r in c["ct"]], n) == I(s)


def test_even_fixture_oracle(golden):
    """The oracle against the reference's even-modulus outcomes (it pins the GPU tests below)."""
    e = golden["even"]
    r = e["researcher"]
    for case in r["cases"]:
        out = O.jl_crypter_aggregate(case["params"], r["round"], r["key"], r["biprime"], r["total"], case["n_expected"])
        assert _bits(out) == _bits([F(v) for v in case["agg"]["ok"]])
    for c in e["crypter"]:
        n, tau = I(c["n"]), I(c["tau"])
        keys = [I(k) for k in c["keys"]]
        for p, enc in enumerate(c["enc"]):
            got = O.jl_encrypt([F(v) for v in c["x"][p]], tau, keys[p], n, len(keys), weight=c["weights"][p])
            assert got == [I(v) for v in enc["ok"]], (c["n"], p)


def test_domain_n_below_one_is_fb624():
    from fedbiomed_amd import _device as D
    from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError

    for n in (0, -4):  # N = 1 is in the domain since round 4 (tests/test_n_one.py)
        with pytest.raises(FedbiomedSecaggCrypterError, match="FB624"):
            D._biprime_limbs(n)
    assert D.fdh_modulus(2**64) == (1, True)  # FDH(2048, 2^64): only odd digests are coprime
    assert D.fdh_modulus(1156 * 1156) == (289, True)


# ------------------------------------------------------------------ GPU: every entry point
@pytest.mark.gpu
def test_node_round_even_biprime_gpu(golden, caplog):
    """reference tests/test_node_secagg.py:207-221: _JLSRound.encrypt -> SecaggCrypter().encrypt(num_nodes=3,
    current_round=1, params=[1.0, 1.0], key=12345, biprime=1156, clipping_range=3, weight=20)."""
    from fedbiomed_amd.secagg import SecaggCrypter

    c = golden["even"]["node_round"]
    with caplog.at_level(logging.WARNING):
        got = SecaggCrypter().encrypt(num_nodes=3, current_round=1, params=[1.0, 1.0], key=12345, biprime=1156,
                                      clipping_range=3, weight=20)
    assert got == [I(v) for v in c["enc"]["ok"]] == [946993]


@pytest.mark.gpu
def test_researcher_aggregate_even_biprime_gpu(golden):
    """reference tests/test_secure_aggregation.py:193-233: aggregate of [[1..5], [1..5]] (5 values) and the
    validation's [[1], [1]] (within 0.03 of -2.9988) with key 1234, biprime 1234, total 100."""
    from fedbiomed_amd.secagg import SecaggCrypter

    r = golden["even"]["researcher"]
    for case in r["cases"]:
        out = SecaggCrypter().aggregate(current_round=1, num_nodes=2, params=case["params"], key=1234, biprime=1234,
                                        total_sample_size=100, clipping_range=None,
                                        num_expected_params=case["n_expected"])
        assert _bits(out) == _bits([F(v) for v in case["agg"]["ok"]])
        assert len(out) == case["n_expected"]
    assert math.isclose(out[0], -2.9988, abs_tol=0.03)


def _sweep_ids():
    from tests.golden_util import load

    return [f"N{I(c['n']).bit_length()}b-P{len(c['keys'])}" for c in load("even.json")["crypter"]]


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(len(_sweep_ids())), ids=_sweep_ids())
def test_even_crypter_sweep_gpu(golden, idx, caplog):
    """SecaggCrypter.encrypt / aggregate over the fixture's even moduli (2..1024 bits, powers of two,
    keys of 8..2040 bits, negative weights, rounds 0..2^64-1): ciphertexts and float64 outputs bit for
    bit, the wrong server key's outcome (floor-division garbage or the reference's error) too."""
    from fedbiomed_amd.secagg import SecaggCrypter

    c = golden["even"]["crypter"][idx]
    n, tau = I(c["n"]), I(c["tau"])
    keys = [I(k) for k in c["keys"]]
    jc = SecaggCrypter()
    encs = []
    with caplog.at_level(logging.WARNING):
        for p, e in enumerate(c["enc"]):
            encs.append(_run(e, lambda p=p: jc.encrypt(num_nodes=len(keys), current_round=tau,
                                                       params=[F(v) for v in c["x"][p]], key=keys[p], biprime=n,
                                                       weight=c["weights"][p])))
            if encs[-1] is not None:
                assert encs[-1] == [I(v) for v in e["ok"]], p
    if "agg" not in c:
        return
    for tag, sk0 in (("agg", -sum(keys)), ("agg_badkey", -sum(keys) + 1)):
        out = _run(c[tag], lambda sk0=sk0: jc.aggregate(current_round=tau, num_nodes=len(keys), params=encs, key=sk0,
                                                        biprime=n, total_sample_size=c["total"],
                                                        num_expected_params=len(c["x"][0])))
        if out is not None:
            assert _bits(out) == _bits([F(v) for v in c[tag]["ok"]]), tag


@pytest.mark.gpu
def test_even_object_api_gpu(golden):
    """UserKey.encrypt (positive and negative keys, plaintexts >= N, >= 2^1024 and negative),
    EncryptedNumber sums, ServerKey.decrypt (the right key, a wrong one, a zero product) on even moduli."""
    from fedbiomed_amd.secagg._jls import EncryptedNumber, ServerKey, UserKey
    from tests.test_jls_api import pp_of

    for c in golden["even"]["object"]:
        n, tau = I(c["n"]), c["tau"]
        pp = pp_of(n)

        keys = [I(k) for k in c["keys"]]
        pts = [I(v) for v in c["pt"]]
        rows = []
        for key, want in zip(keys, c["ct"]):
            got = UserKey(pp, key).encrypt(pts, tau)
            assert got == [I(v) for v in want], (c["n"], key)
            rows.append([EncryptedNumber(pp, v) for v in got])
        summed = [sum(ep) for ep in zip(*rows)]
        assert [s.ciphertext for s in summed] == [I(v) for v in c["sum"]]
        assert ServerKey(pp, -sum(keys)).decrypt(summed, tau) == [I(v) for v in c["dec"]["ok"]]
        assert ServerKey(pp, -sum(keys) + 3).decrypt(summed, tau) == [I(v) for v in c["dec_badkey"]["ok"]]
        zero = [EncryptedNumber(pp, 0), EncryptedNumber(pp, n * n)]
        assert ServerKey(pp, -sum(keys)).decrypt(zero, tau) == [I(v) for v in c["dec_zero"]["ok"]] == [n - 1] * 2


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [2, 3, 17, 33, 64, 65, 300, 512, 1000, 1024])
def test_even_random_moduli_gpu(bits):
    """Random even moduli of every size class through the C-ABI (raw UserKey.encrypt of int64
    plaintexts, keys of either sign, the server decrypt of the product) against the oracle."""
    import torch

    from fedbiomed_amd import _device as D

    rng = random.Random(5000 + bits)
    N = (rng.getrandbits(bits) | (1 << (bits - 1))) & ~1
    if bits == 65:
        N = 2**64  # a power of two: FDH needs odd digests only, m^2 = 1
    n, P, tau = 45, 3, rng.getrandbits(64)
    pts = [rng.getrandbits(63) for _ in range(n)]
    keys = [rng.getrandbits(rng.choice([1, 40, 700, 2040])) * rng.choice([1, -1]) for _ in range(P)]
    keys[2] = 0 if bits == 17 else keys[2]
    dev = D.device()
    n2 = N * N
    # N a power of two: a ciphertext whose 7 FDH digests all end even has no coprime r -- the
    # reference's OverflowError (counter.to_bytes(1) past 255, _jls.py:742-760), raised here too;
    # the ciphertexts before the first such index are then compared
    bad = []
    for k in range(n):
        try:
            O.fdh((k << 512) | tau, n2)
        except OverflowError:
            bad.append(k)
    if bad:
        with pytest.raises(OverflowError):
            D.jl_encrypt(torch.tensor(pts, dtype=torch.int64, device=dev), N, keys[0], tau, P, slot=(100, 1))
        n = bad[0]
        pts = pts[:n]
    x = torch.tensor(pts, dtype=torch.int64, device=dev)
    cts = []
    for key in keys:
        got = D.jl_encrypt(x, N, key, tau, P, slot=(100, 1))
        want = [((N * pt + 1) % n2) * O.powmod(O.fdh((k << 512) | tau, n2), key, n2) % n2 for k, pt in enumerate(pts)]
        assert D.limbs_to_ints(got.cpu().numpy()) == want, (bits, key)
        cts.append(got)
    sk0 = -sum(keys)
    _, sums = D.jl_aggregate(torch.stack(cts), N, sk0, tau, n, 1, want_out=False, want_sums=True, slot=(100, 1))
    s = sums.cpu().numpy().view(np.uint64)
    got = [int(a) | (int(b) << 64) for a, b in s]
    ints = [D.limbs_to_ints(c.cpu().numpy()) for c in cts]
    want = []
    for k in range(n):
        prod = 1
        for row in ints:
            prod = prod * row[k] % n2
        v = prod * O.powmod(O.fdh((k << 512) | tau, n2), sk0, n2) % n2
        want.append(((v - 1) // N) % N)
    assert got == want


@pytest.mark.gpu
def test_generic_engine_equals_montgomery_engines_gpu():
    """On odd moduli the generic engine (jl_engine("generic")) and the Montgomery engines give the
    same ciphertexts and sums bit for bit: the 1024-bit benchmark biprime, 2040-bit keys of either
    sign, a full crypter encrypt + aggregate of 3 parties, plus a decryption factor alone."""
    import torch

    from fedbiomed_amd import _device as D
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    rng = np.random.default_rng(9)
    n, P, tau = 3 * 31 * 20 + 7, 3, 5
    xs = [torch.tensor(rng.standard_normal(n) * 0.5, dtype=torch.float32, device=dev) for _ in range(P)]
    keys = [W.jl_user_key(p) for p in range(P)]
    keys[1] = -keys[1]
    jc = SecaggCrypter()
    res = {}
    for eng in ("auto", "generic"):
        with D.jl_engine(eng):
            cts = torch.stack([jc.encrypt_tensor(P, tau, x, k, W.BIPRIME0, weight=3 + p)
                               for p, (x, k) in enumerate(zip(xs, keys))])
            out, sums = jc.aggregate_tensor(tau, cts, -sum(keys), W.BIPRIME0, 3 * P + 3, num_expected_params=n,
                                            want_sums=True)
            f = jc.decrypt_factor_tensor(tau, 40, -sum(keys), W.BIPRIME0, ct_offset=11)
            torch.cuda.synchronize()
            res[eng] = (cts.cpu(), out.cpu(), sums.cpu(), f.cpu())
    for a, b in zip(res["auto"], res["generic"]):
        assert torch.equal(a, b)
