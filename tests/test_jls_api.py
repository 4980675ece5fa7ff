"""The JoyeLibert object API (fedbiomed_amd/secagg/_jls.py) against the reference's own
classes: the reference's tests (tests/test_joye_libert.py) restated for the mirror, and the
golden outputs of the reference classes (tests/golden/jls_api.json, tools/gen_golden.py
gen_jls_api) -- FDH over odd, even and non-square moduli, _populate_tau, UserKey.encrypt on raw
plaintexts, EncryptedNumber sums, ServerKey.decrypt, JoyeLibert.protect / aggregate, VES.
Every integer output is compared bit-exactly.  The argument checks that precede any device
call run on the CPU; everything else runs the HIP path (`gpu`)."""

import math
import random

import pytest

from fedbiomed_amd.constants import SAParameters
from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError
from fedbiomed_amd.secagg._jls import (
    FDH,
    VES,
    BaseKey,
    EncryptedNumber,
    JoyeLibert,
    PublicParam,
    ServerKey,
    UserKey,
)
from tests.golden_util import I

P_REF = int("7801876574383880214548650574033350741129913580793719706746361606042541080141291132224899113047934760"
            "791108387050756752894517232516965892712015132079112571")
Q_REF = int("7755946847853454424709929267431997195175500554762787715247111385596652741022399320865688002114973453"
            "057088521173384791077635017567166681500095602864712097")


def pp_of(n: int) -> PublicParam:
    return PublicParam(n_modulus=n, bits=SAParameters.KEY_SIZE // 2, hashing_function=FDH(SAParameters.KEY_SIZE, n * n).H)


def _expect(outcome, fn):
    """Run fn and compare with a golden {"ok": ...} / {"error": type, "msg": ...} outcome."""
    if "error" in outcome:
        with pytest.raises(Exception) as ei:
            fn()
        assert type(ei.value).__name__ == outcome["error"], (ei.value, outcome)
        assert str(ei.value) == outcome["msg"]
    else:
        return fn()


# ------------------------------------------------------------------ argument checks (CPU)
def test_fdh_init_types():
    """reference test_joye_libert.py:19-32 (an int modulus is accepted: gmpy2 is not a dependency)"""
    with pytest.raises(TypeError):
        FDH(bits_size=SAParameters.KEY_SIZE, n_modulus="1234")
    with pytest.raises(TypeError):
        FDH(bits_size="not-int", n_modulus=12123)
    with pytest.raises(TypeError):
        FDH(bits_size=SAParameters.KEY_SIZE, n_modulus=1.5)
    FDH(bits_size=SAParameters.KEY_SIZE, n_modulus=12123)


def test_public_param_equality_getters():
    """reference test_joye_libert.py:48-81"""
    pp1, pp2 = pp_of(123456), pp_of(123456789)
    assert not pp1 == pp2
    assert pp1 == pp1
    assert pp1.bits == SAParameters.KEY_SIZE // 2
    assert pp1.n_modulus == 123456
    assert pp1.n_square == 123456 * 123456
    assert repr(pp1).startswith("<PublicParam (N=12345...23456")


def test_base_key():
    """reference test_joye_libert.py:147-193 (hash, equality, types)"""
    pp = pp_of(123457)
    bk = BaseKey(public_param=pp, key=191919191919191)
    assert bk.public_param == pp
    assert repr(bk).startswith("<ServerKey 0x")
    assert hash(bk) == 191919191919191
    assert bk == bk
    assert not bk == BaseKey(public_param=pp_of(123457), key=19191919191919121)
    with pytest.raises(TypeError):
        bk == 10  # noqa: B015
    with pytest.raises(TypeError):
        UserKey(pp, 10) == ServerKey(pp, 10)  # noqa: B015


def test_argument_errors_match_reference(golden):
    """The error outcomes of the reference's own checks (jls_api.json "errors"), raised before
    any device work."""
    e = golden["jls_api"]["errors"]
    pp = pp_of(P_REF * Q_REF)
    uk, jl = UserKey(pp, 10), JoyeLibert()
    _expect(e["protect_bad_key"], lambda: jl.protect(pp, "in-valid-user-key", 1, [1], 2))
    _expect(e["protect_bad_param"], lambda: jl.protect(pp_of(1111), uk, 1, [1], 2))
    _expect(e["protect_bad_x"], lambda: jl.protect(pp, uk, 1, "invalid-plaintext", 2))
    _expect(e["aggregate_bad_key"], lambda: jl.aggregate(uk, 1, [[1]], 1))
    _expect(e["aggregate_empty"], lambda: jl.aggregate(ServerKey(pp, -10), 1, [], 1))
    _expect(e["aggregate_not_nested"], lambda: jl.aggregate(ServerKey(pp, -10), 1, [1, 2], 1))
    _expect(e["encrypt_not_list"], lambda: uk.encrypt("not-a-list", 1))
    _expect(e["decrypt_not_list"], lambda: ServerKey(pp, -10).decrypt("x", 1))
    _expect(e["decrypt_not_en"], lambda: ServerKey(pp, -10).decrypt([1, 2], 1))
    _expect(e["key_not_int"], lambda: UserKey(pp, 1.5))
    _expect(e["en_plus_int"], lambda: EncryptedNumber(pp, 10) + 15)
    _expect(e["en_param_mismatch"], lambda: EncryptedNumber(pp, 10) + EncryptedNumber(pp_of(987654123), 10))
    _expect(e["fdh_bits_str"], lambda: FDH("not-int", 12123))
    _expect(e["fdh_mod_str"], lambda: FDH(2048, "1234"))
    with pytest.raises(TypeError):  # aggregate of ints: ServerKey.decrypt's type check
        jl.aggregate(ServerKey(pp, -10), 1, [[1, 2]], 2)


def test_encrypted_number_sums_are_lazy():
    """Sums keep their operands (no arithmetic until the ciphertext is read); sum() and the
    parameter check behave as the reference's."""
    pp = pp_of(123457)
    en = EncryptedNumber(param=pp, ciphertext=10)
    s = sum([en, en, en])
    assert s._terms == (10, 10, 10) and s._value is None
    assert (0 + en) is en
    with pytest.raises(ValueError):
        en + EncryptedNumber(pp_of(987654123), 10)


def test_domain_restrictions_raise_fb624():
    pp = pp_of(123457)
    # (FDH of any other bits_size: on the device since round 4 -- tests/test_fdh_bits.py)
    with pytest.raises(FedbiomedSecaggCrypterError, match="FB624"):
        UserKey(pp_of(0), 3).encrypt([1], 1)  # N = 0 (every N >= 1 is in the domain: tests/test_n_one.py)
    # (rounds of 2^512 and more, FDH.H of any t < 2^8192: on the device since ABI 3 -- tests/test_caller_flows.py)
    with pytest.raises(OverflowError):
        UserKey(pp, 3).encrypt([1], 2**8192)  # int(t).to_bytes(1024) of the reference
    # (delta^2 != 1 (mod N): on the device since round 5 -- tests/test_decrypt_delta.py)
    with pytest.raises(ZeroDivisionError):
        ServerKey(pp, -20).decrypt([EncryptedNumber(pp, 5)], 1, delta=0)  # invert(0) as the reference
    # a non-FDH hashing function is the caller's own callable: _populate_tau calls it per t
    assert BaseKey(PublicParam(123457, 1024, lambda t: t + 1), 1)._populate_tau(3, 2) == [4, (1 << 512 | 3) + 1]


# ------------------------------------------------------------------ device parity (GPU)
@pytest.mark.gpu
def test_even_modulus_user_encrypt(golden):
    """An even N (123456) is encrypted as the reference does (the generic engine, csrc/fbm_gen.hip);
    rounds 2 and earlier refused it with FB624."""
    assert UserKey(pp_of(123456), 3).encrypt([1], 1) == [I(v) for v in golden["even"]["user_encrypt_123456"]]


@pytest.mark.gpu
def test_fdh_golden(golden):
    for case in golden["jls_api"]["fdh"]:
        fdh = FDH(2048, I(case["m"]))
        for t, h in zip(case["t"], case["h"]):
            if "ok" in h:
                assert fdh.H(I(t)) == I(h["ok"]), (case["m"], t)
            else:
                with pytest.raises(OverflowError):
                    fdh.H(I(t))


@pytest.mark.gpu
def test_fdh_reference_test_values():
    """reference test_joye_libert.py:34-45"""
    fdh = FDH(bits_size=SAParameters.KEY_SIZE, n_modulus=12345)
    r1 = fdh.H(10)
    assert r1 != 0 and isinstance(r1, int)
    assert fdh.H(10) == r1
    assert pp_of(123456).hashing_function(10) != 0  # test_public_param_03: even modulus


@pytest.mark.gpu
def test_populate_tau_golden(golden):
    for case in golden["jls_api"]["populate_tau"]:
        bk = BaseKey(pp_of(I(case["n"])), 191919191919191)
        got = _expect(case["h"], lambda bk=bk, case=case: bk._populate_tau(tau=case["tau"], len_=case["len"]))
        if "ok" in case["h"]:
            assert got == [I(h) for h in case["h"]["ok"]]
            if I(case["n"]) == 123457:  # reference test_joye_libert.py:188-193 (no gcd retry there)
                assert all(r.bit_length() <= SAParameters.KEY_SIZE // 8 for r in got)


@pytest.mark.gpu
def test_user_key_encrypt_golden(golden):
    for case in golden["jls_api"]["user_encrypt"]:
        uk = UserKey(pp_of(I(case["n"])), I(case["key"]))
        got = uk.encrypt([I(v) for v in case["pt"]], case["tau"])
        assert got == [I(c) for c in case["ct"]], case["n"]
    uk = UserKey(pp_of(123457), 191919191919191)  # reference test_joye_libert.py:211-222
    en = uk.encrypt(plaintext=[10, 10, 10], tau=1)
    assert isinstance(en, list) and len(en) == 3
    assert uk.encrypt([], 1) == []


@pytest.mark.gpu
def test_encrypted_number_sums_golden(golden):
    pp = pp_of(123457)  # reference test_joye_libert.py:99-124
    en = EncryptedNumber(param=pp, ciphertext=10)
    assert (en + en).ciphertext == 100
    assert (en + en + en + en).ciphertext == 10000
    assert [s.ciphertext for s in [sum(ep) for ep in zip(*[[en] * 3, [en] * 3])]] == [100, 100, 100]
    acc = en
    acc += en
    assert acc.ciphertext == 100 and repr(acc) == "<EncryptedNumber 100...100>"
    for case in golden["jls_api"]["sums"]:
        ppc = pp_of(I(case["n"]))
        total = sum(EncryptedNumber(ppc, I(c)) for c in case["cts"])
        assert total.ciphertext == I(case["sum"])


@pytest.mark.gpu
def test_server_key_decrypt_golden(golden):
    n = 123457  # reference test_joye_libert.py:225-252
    pp = pp_of(n)
    en_1 = [EncryptedNumber(pp, c) for c in UserKey(pp, 10).encrypt([10, 10, 10], tau=1)]
    en_2 = [EncryptedNumber(pp, c) for c in UserKey(pp, 10).encrypt([10, 10, 10], tau=1)]
    assert ServerKey(pp, -20).decrypt([sum(en) for en in zip(*[en_1, en_2])], tau=1) == [20, 20, 20]
    for case in golden["jls_api"]["decrypt"]:
        ppc = pp_of(I(case["n"]))
        keys = [I(k) for k in case["keys"]]
        encs = [[EncryptedNumber(ppc, I(c)) for c in row] for row in case["cts"]]
        summed = [sum(ep) for ep in zip(*encs)]  # lazy: the products run inside decrypt
        assert ServerKey(ppc, -sum(keys)).decrypt(summed, case["tau"], delta=case["delta"]) == \
            [I(v) for v in case["dec"]]
        assert ServerKey(ppc, -sum(keys) + 1).decrypt(summed, case["tau"]) == [I(v) for v in case["dec_badkey"]]
        materialised = [EncryptedNumber(ppc, s.ciphertext) for s in summed]  # one product per number
        assert ServerKey(ppc, -sum(keys)).decrypt(materialised, case["tau"]) == [I(v) for v in case["dec"]]


@pytest.mark.gpu
def test_joye_libert_protect_aggregate_golden(golden):
    g = golden["jls_api"]
    for case, agg in zip(g["protect"], g["aggregate"]):
        n, keys = I(case["n"]), [I(k) for k in case["keys"]]
        target = I(case["target"]) if case["target"] else None
        pp = pp_of(n)
        jl = JoyeLibert(target_range=target)
        x = [I(v) for v in case["x"]]
        prot = [jl.protect(pp, UserKey(pp, k), case["tau"], list(x), len(keys)) for k in keys]
        assert prot == [[I(c) for c in row] for row in case["ct"]]
        encs = [[EncryptedNumber(pp, c) for c in row] for row in prot]
        for ne, res in zip(agg["n_expected"], agg["out"]):
            assert jl.aggregate(ServerKey(pp, -sum(keys)), case["tau"], encs, ne) == [I(v) for v in res["ok"]]


@pytest.mark.gpu
def test_joye_libert_reference_flow():
    """reference test_joye_libert.py:255-421"""
    pp = pp_of(P_REF * Q_REF)
    jl, uk1, uk2, sk = JoyeLibert(), UserKey(pp, 10), UserKey(pp, 10), ServerKey(pp, -20)
    assert len(jl.protect(public_param=pp, user_key=uk1, tau=1, x_u_tau=[10, 10, 10], n_users=2)) == 1
    ref_pt = list(range(11, 28)) * 5
    assert len(jl.protect(public_param=pp, user_key=uk1, tau=1, x_u_tau=ref_pt, n_users=2)) == 3
    for plaintext in ([10, 10, 10], [0, 5, 20, 0]):
        en_1 = [EncryptedNumber(pp, int(e)) for e in jl.protect(pp, uk1, 1, plaintext, 2)]
        en_2 = [EncryptedNumber(pp, int(e)) for e in jl.protect(pp, uk2, 1, plaintext, 2)]
        agg = jl.aggregate(sk_0=sk, tau=1, list_y_u_tau=[en_1, en_2], num_expected_params=len(plaintext))
        assert agg == [2 * el for el in plaintext]


@pytest.mark.gpu
def test_ves_golden(golden):
    for case in golden["jls_api"]["ves"]:
        ves = VES(case["ptsize"], case["valuesize"])
        V = [I(v) for v in case["V"]]
        E = [I(e) for e in case["E"]]
        # (a value wider than its slot may spill past bit 1024: the general kernels since round 4)
        assert ves.encode(list(V), case["add_ops"]) == E
        assert ves.decode(E, case["add_ops"], case["v_expected"]) == [I(v) for v in case["D"]]


@pytest.mark.gpu
def test_random_protect_aggregate_vs_oracle():
    """A 3-user round of 2 000 random values per user on biprime0, checked against the oracle."""
    from fedbiomed_amd import workload as W
    from oracle import secagg_oracle as O

    rng = random.Random(5)
    n = W.BIPRIME0
    pp = pp_of(n)
    keys = [W.jl_user_key(u) for u in range(3)]
    xs = [[rng.getrandbits(30) for _ in range(2000)] for _ in keys]
    jl = JoyeLibert()
    prot = [jl.protect(pp, UserKey(pp, k), 9, x, 3) for k, x in zip(keys, xs)]
    for u in (0, 2):  # sampled ciphertexts vs the oracle
        ks = sorted(rng.sample(range(len(prot[u])), 6))
        cr = O.jl_slot(None, 3)[1]
        ref = O.jl_encrypt_ints(xs[u][:(ks[-1] + 1) * cr], 9, keys[u], n, 3)
        assert [prot[u][k] for k in ks] == [ref[k] for k in ks]
    encs = [[EncryptedNumber(pp, c) for c in row] for row in prot]
    assert jl.aggregate(ServerKey(pp, -sum(keys)), 9, encs, 2000) == [sum(v) for v in zip(*xs)]


def test_crypter_public_param_helpers():
    """reference test_secagg_crypter.py:23-47"""
    from fedbiomed_amd.secagg import SecaggCrypter

    pp = SecaggCrypter._setup_public_param(biprime=12345)
    assert isinstance(pp, PublicParam) and pp.n_modulus == 12345 and pp.bits == 1024
    enc = SecaggCrypter._convert_to_encrypted_number([[1, 2, 3, 4], [1, 2, 3, 4], [1, 2, 3, 4]], pp)
    assert isinstance(enc[0][0], EncryptedNumber) and isinstance(enc[2][3], EncryptedNumber)
    assert enc[0][0].ciphertext == 1 and enc[2][3].ciphertext == 4


@pytest.mark.gpu
def test_decrypt_of_zero_product():
    """A product = 0 mod N^2 (a zero ciphertext): ((0 - 1) // N) % N = N - 1, as Python computes it
    in ServerKey.decrypt (_jls.py:553-554) -- through the object API and the crypter's combine."""
    from fedbiomed_amd import workload as W
    from oracle import secagg_oracle as O

    for n in (123457, W.BIPRIME0):
        pp = pp_of(n)
        cts = [0, n * n, 5, 0]
        got = ServerKey(pp, -20).decrypt([EncryptedNumber(pp, c) for c in cts], tau=3)
        assert got == O.jl_server_decrypt(cts, 3, -20, n) and got[0] == n - 1
        en = [[EncryptedNumber(pp, c) for c in cts], [EncryptedNumber(pp, 7)] * 4]
        jl = JoyeLibert()
        es, cr = jl._vector_encoder._get_elements_size_and_compression_ratio(2)
        xs = O.jl_server_decrypt([c * 7 % (n * n) for c in cts], 3, -20, n)
        assert jl.aggregate(ServerKey(pp, -20), 3, en, 4 * cr) == O.ves_decode(xs, es, cr, 4 * cr)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [2, 5, 17, 64, 129, 511, 1000, 1024])
def test_random_moduli_object_api_vs_oracle(bits):
    """UserKey.encrypt / EncryptedNumber sums / ServerKey.decrypt on random odd moduli (FDH
    retries on the small ones) with keys of both signs and plaintexts at the edges (0, N - 1,
    N, 2^1024 - 1, negative), against the oracle."""
    from oracle import secagg_oracle as O

    rng = random.Random(1000 + bits)
    n = rng.getrandbits(bits) | 1 | (1 << (bits - 1))
    if n < 3:
        n = 3
    pp = pp_of(n)
    keys = [rng.getrandbits(rng.choice([1, 64, 2040])) * rng.choice([1, -1]) for _ in range(3)]
    pts = [0, n - 1, n, 2**1024 - 1, -7, 1] + [rng.getrandbits(1024) for _ in range(10)]
    tau = rng.getrandbits(64)
    try:
        ref = [O.jl_user_encrypt(pts, tau, k, n) for k in keys]
    except (OverflowError, ValueError) as e:  # FDH exhausted / H not invertible for a negative key
        with pytest.raises(type(e) if isinstance(e, OverflowError) else (ZeroDivisionError, ValueError)):
            for k in keys:
                UserKey(pp, k).encrypt(pts, tau)
        return
    got = [UserKey(pp, k).encrypt(list(pts), tau) for k in keys]
    assert got == ref
    summed = [sum(ep) for ep in zip(*[[EncryptedNumber(pp, c) for c in row] for row in got])]
    products = [math.prod(col) % (n * n) for col in zip(*ref)]
    assert [s.ciphertext for s in summed[:4]] == products[:4]  # materialised one by one on the device
    sk = -sum(keys)
    try:
        want = O.jl_server_decrypt(products, tau, sk, n)
    except ValueError:  # the server power is not invertible mod N^2
        with pytest.raises(ZeroDivisionError):
            ServerKey(pp, sk).decrypt(summed, tau)
        return
    assert ServerKey(pp, sk).decrypt(summed, tau) == want


@pytest.mark.gpu
def test_crypter_average_weighting_helpers():
    """reference test_secagg_crypter.py:49-120 (_apply_average / _apply_weighting, on the device),
    plus Python's int/int rounding above 2^53 and weights up to 2^17."""
    from fedbiomed_amd.secagg import SecaggCrypter

    sc = SecaggCrypter()
    assert sc._apply_average([4, 8, 12], 2) == [v / 2 for v in [4, 8, 12]]
    big = [2**53 + 1, 2**64 + 3, 2**127 - 1, 3, 0, 10**30 + 7]
    assert sc._apply_average(big, 7) == [v / 7 for v in big]
    assert sc._apply_average(big, 2**64 - 1) == [v / (2**64 - 1) for v in big]
    for vector in ([-1], [1, 1, -1], [-1, 1, 1], [1, -1, 1]):
        with pytest.raises(FedbiomedSecaggCrypterError):
            sc._apply_average(vector, 2)
    assert sc._apply_weighting([4, 8, 12], 2) == [8, 16, 24]
    assert sc._apply_weighting([0, 8191, 5], 2**17 - 1) == [0, 8191 * (2**17 - 1), 5 * (2**17 - 1)]
    T = SAParameters.TARGET_RANGE
    for vector in ([-1], [1, 1, -1], [-1, 1, 1], [1, -1, 1], [T], [2 * T], [0, T, 0], [0, 0, T]):
        with pytest.raises(FedbiomedSecaggCrypterError):
            sc._apply_weighting(vector, 2)
    with pytest.raises(FedbiomedSecaggCrypterError):
        sc._apply_weighting([T], 2)
    assert sc._apply_weighting([T], 2, target_range=SAParameters.FA_TARGET_RANGE) == [2 * T]
    with pytest.raises(FedbiomedSecaggCrypterError):
        sc._apply_weighting([SAParameters.FA_TARGET_RANGE], 2, target_range=SAParameters.FA_TARGET_RANGE)


@pytest.mark.gpu
def test_object_api_equals_fused_crypter_at_config2():
    """Config 2 (JL, 100k elements, 4 parties): SecaggCrypter.encrypt (fused quantise + weight + pack +
    encrypt) equals JoyeLibert.protect on the reference's quantize() * weight integers, and
    JoyeLibert.aggregate's decoded sums equal the crypter's sums (device tensors, one call each)."""
    import numpy as np
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter
    from fedbiomed_amd.utils import quantize

    n, P, tau = 100_000, 4, 5
    bp = W.BIPRIME0
    keys = [W.jl_user_key(p) for p in range(P)]
    xs = [[float(v) for v in W.party_params(p, n)] for p in range(P)]
    ws = [W.party_weight(p) for p in range(P)]
    sc, jl = SecaggCrypter(), JoyeLibert()
    pp = SecaggCrypter._setup_public_param(bp)
    fused = [sc.encrypt(P, tau, xs[p], keys[p], bp, weight=ws[p]) for p in range(P)]
    ints = [[q * ws[p] for q in quantize(xs[p])] for p in range(P)]
    obj = [jl.protect(pp, UserKey(pp, keys[p]), tau, ints[p], P) for p in range(P)]
    assert obj == fused
    sums = jl.aggregate(ServerKey(pp, -sum(keys)), tau, SecaggCrypter._convert_to_encrypted_number(obj, pp), n)
    assert sums == [sum(col) for col in zip(*ints)]
    cts = torch.stack([torch.from_numpy(D.ints_to_limbs(row).view(np.int32)) for row in fused]).cuda()
    _, dev_sums = sc.aggregate_tensor(tau, cts, -sum(keys), bp, sum(ws), num_expected_params=n, want_sums=True)
    s = dev_sums.cpu().numpy().view("<u8")
    assert [int(lo) | (int(hi) << 64) for lo, hi in s.tolist()] == sums
