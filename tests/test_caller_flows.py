"""The reference's caller-level secagg flows, pinned by the reference crypter's
own outputs on their crypter-level inputs (tests/golden/caller_flows.json, tools/gen_golden.py
gen_caller_flows; the callers' tests themselves need declearn / tinydb / ..., absent here: SURVEY 4):

* LOM -- tests/test_secure_aggregation.py:383-426 (create_protected_vector: quantize -> multiply by 5 ->
  LOM(nonce).protect per node), :487-519 (LomSecureAggregation.aggregate -> SecaggLomCrypter.aggregate,
  total_sample_size 5, clip 1000: the test's own expectation round(out) == sum + 2 clip), :520-558 (an
  explicit clip of 2000); the reference draws its nonce with token_bytes: fixed nonces here;
* JL -- tests/test_optimizer_secagg.py:513-631 (the Scaffold aux-var flow: SecaggCrypter().encrypt of a
  Linear(4, 2) model's 10 weights and 10 corrections, clip 3, weight 5 or None; the same ciphertexts from
  2 / 3 / 5 / 8 / 10 nodes, rounds 1..4, aggregate with -(key x nodes), num_expected_params 10, that
  test's biprime); seeded vectors and keys where the test draws random ones.

CPU: the oracle reproduces every fixture value.  GPU: the drop-in (fedbiomed_amd.utils,
fedbiomed_amd.secagg) reproduces them bit for bit."""

import json
import os
import struct

import numpy as np
import pytest

from oracle import secagg_oracle as O

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "caller_flows.json")))


def I(s):  # noqa: E743
    return int(s, 16)


def F(s):
    return struct.unpack(">d", bytes.fromhex(s[2:]))[0]


def _params(p):
    return [F(v) if isinstance(v, str) else v for v in p]


def _bits(xs):
    return np.asarray(xs, dtype=np.float64).view(np.uint64).tolist()


def test_oracle_lom_caller_flow():
    for c in FIX["lom"]:
        nonce = bytes.fromhex(c["nonce"])
        qs = [[int(v) * c["weight"] for v in O.quantize(np.asarray(_params(p), np.float64), c["clip"])]
              for p in c["params"]]
        assert qs == [[I(v) for v in x] for x in c["quantized"]]
        sec = {u: {v: b"\x02" * 32 for v in c["parties"] if v != u} for u in c["parties"]}
        pv = [O.lom_protect(u, sec[u], c["round"], x, c["parties"], nonce) for u, x in zip(c["parties"], qs)]
        assert [[int(v) for v in y] for y in pv] == [[I(v) for v in y] for y in c["protected"]]
        agg = O.lom_crypter_aggregate(pv, c["total_sample_size"], c["clip"])
        assert _bits(agg) == _bits([F(v) for v in c["agg"]])


def test_reference_expectation_of_the_lom_flow():
    """test_secure_aggregation.py:513-519: round(out) == column sum + 2 clip; :552-558 (clip 2000): within
    atol 2 of it -- the reference's own checks, on the reference's outputs."""
    for c, rounded in zip(FIX["lom"][:2], (True, False)):
        want = np.sum([_params(p) for p in c["params"]], axis=0) + 2 * c["clip"]
        got = [F(v) for v in c["agg"]]
        if rounded:
            assert all(np.isclose(np.round(g), w) for g, w in zip(got, want))
        else:
            assert all(np.isclose(g, w, atol=2) for g, w in zip(got, want))


def test_oracle_jl_auxvar_flow():
    N = I(FIX["jl_auxvar_biprime"])
    for c in FIX["jl_auxvar"][::7]:  # a spread of the 40 cases (every node count, round and weighting)
        key, n, rnd = I(c["key"]), c["num_nodes"], c["round"]
        for name in ("aux", "weights"):
            d = c[name]
            enc = O.jl_encrypt([F(v) for v in d["x"]], rnd, key, N, n, clip=3, weight=c["weight"])
            assert enc == [I(v) for v in d["enc"]]
            dec = O.jl_crypter_aggregate([enc] * n, rnd, -(key * n), N, c["total_sample_size"], 10, clip=3)
            assert _bits(dec) == _bits([F(v) for v in d["dec"]])


@pytest.mark.gpu
def test_drop_in_lom_caller_flow():
    from fedbiomed_amd.secagg import LOM, SecaggLomCrypter
    from fedbiomed_amd.utils import multiply, quantize

    for c in FIX["lom"]:
        nonce = bytes.fromhex(c["nonce"])
        qs = [multiply(quantize(_params(p), c["clip"]), c["weight"]) for p in c["params"]]
        assert qs == [[I(v) for v in x] for x in c["quantized"]]
        sec = {u: {v: b"\x02" * 32 for v in c["parties"] if v != u} for u in c["parties"]}
        pv = [LOM(nonce=nonce).protect(u, sec[u], c["round"], x, c["parties"]) for u, x in zip(c["parties"], qs)]
        assert pv == [[I(v) for v in y] for y in c["protected"]]
        agg = SecaggLomCrypter().aggregate(params=pv, total_sample_size=c["total_sample_size"],
                                           clipping_range=c["clip"], target_range=None)
        assert _bits(agg) == _bits([F(v) for v in c["agg"]])


@pytest.mark.gpu
def test_drop_in_jl_auxvar_flow():
    from fedbiomed_amd.secagg import SecaggCrypter

    N = I(FIX["jl_auxvar_biprime"])
    for c in FIX["jl_auxvar"]:
        key, n, rnd = I(c["key"]), c["num_nodes"], c["round"]
        for name in ("aux", "weights"):
            d = c[name]
            enc = SecaggCrypter().encrypt(params=[F(v) for v in d["x"]], key=key, num_nodes=n, current_round=rnd,
                                          biprime=N, clipping_range=3, weight=c["weight"])
            assert enc == [I(v) for v in d["enc"]], (n, rnd, name)
            dec = SecaggCrypter().aggregate(params=[enc] * n, key=-(key * n), total_sample_size=c["total_sample_size"],
                                            num_nodes=n, current_round=rnd, biprime=N, clipping_range=3,
                                            num_expected_params=10)
            assert _bits(dec) == _bits([F(v) for v in d["dec"]]), (n, rnd, name)


def test_oracle_big_rounds():
    """Rounds of 2^512 and more (ABI 3): the reference ORs them into t = (k << 512) | tau and hashes t
    whole; the oracle's FDH / encrypt reproduce its values (they pin the GPU test below)."""
    from fedbiomed_amd import workload as W

    n2 = W.BIPRIME0 ** 2
    for c in FIX["big_fdh"]:
        assert O.fdh(I(c["t"]), n2) == I(c["h"])
    for r in FIX["big_rounds"][::3]:
        tau, keys = I(r["tau"]), [I(k) for k in r["keys"]]
        enc = O.jl_encrypt([F(v) for v in r["x"][0]], tau, keys[0], W.BIPRIME0, 2, weight=3)
        assert enc == [I(v) for v in r["enc"][0]]
    assert FIX["round_overflow"] == {"error": "OverflowError", "msg": "int too big to convert"}


def test_round_limbs_abi3():
    from fedbiomed_amd import _device as D, _native

    assert _native.TAU_LIMBS == 256
    assert D._check_round(2**8192 - 1).tolist() == [0xFFFFFFFF] * 256
    assert D._check_round(2**512 + 7).tolist() == [7] + [0] * 15 + [1] + [0] * 239
    with pytest.raises(OverflowError, match="int too big to convert"):
        D._check_round(2**8192)
    with pytest.raises(OverflowError):
        D._check_round(-1)


@pytest.mark.gpu
def test_drop_in_big_rounds():
    """SecaggCrypter.encrypt / aggregate at rounds 2^512 ... 2^8192 - 1 (k's bits ORed with the round's,
    the round's bits 1024.. in FDH's leading blocks: a per-call midstate) and FDH.H of any t < 2^8192:
    the reference's values bit for bit; 2^8192 is its OverflowError."""
    from fedbiomed_amd import workload as W
    from fedbiomed_amd.secagg import SecaggCrypter
    from fedbiomed_amd.secagg._jls import FDH

    jc = SecaggCrypter()
    for r in FIX["big_rounds"]:
        tau, keys = I(r["tau"]), [I(k) for k in r["keys"]]
        enc = [jc.encrypt(num_nodes=2, current_round=tau, params=[F(v) for v in x], key=k, biprime=W.BIPRIME0,
                          weight=3) for x, k in zip(r["x"], keys)]
        assert enc == [[I(v) for v in e] for e in r["enc"]], r["tau"][:12]
        out = jc.aggregate(current_round=tau, num_nodes=2, params=enc, key=-sum(keys), biprime=W.BIPRIME0,
                           total_sample_size=6, num_expected_params=70)
        assert _bits(out) == _bits([F(v) for v in r["agg"]])
    n2 = W.BIPRIME0 ** 2
    for c in FIX["big_fdh"]:
        assert FDH(2048, n2).H(I(c["t"])) == I(c["h"])
    with pytest.raises(OverflowError, match="int too big to convert"):
        jc.encrypt(num_nodes=2, current_round=2**8192, params=[0.5], key=5, biprime=W.BIPRIME0)
