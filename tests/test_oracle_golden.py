"""Pins the CPU oracle (oracle/secagg_oracle.py) to golden vectors produced by the
reference Fed-BioMed implementation itself.  CPU only."""

import math

import numpy as np
import pytest

from oracle import secagg_oracle as O
from tests.golden_util import F, I, fbits


def test_quantize_golden(golden):
    for case in golden["quantize"]["quantize"]:
        x = np.array([F(v) for v in case["x"]])
        got = O.quantize(x, case["clip"], I(case["target"]))
        exp = [I(v) for v in case["q"]]
        assert [int(v) for v in got] == exp, (case["clip"], case["target"])


def test_reverse_quantize_golden(golden):
    for case in golden["quantize"]["reverse_quantize"]:
        v = [F(x) for x in case["v"]] if "v" in case else [I(x) for x in case["v_int"]]
        got = O.reverse_quantize(v, case["clip"], I(case["target"]))
        assert [fbits(a) for a in got] == [s[2:] for s in case["out"]]


def test_true_div_golden(golden):
    for case in golden["quantize"]["true_div"]:
        assert fbits(O.apply_average([I(case["e"])], I(case["w"]))[0]) == case["q"][2:]


def test_prf_golden(golden):
    for case in golden["lom"]["prf"]:
        nonce = bytes.fromhex(case["nonce"])
        seed = O.prf_eval_key(bytes.fromhex(case["secret"]), nonce, case["tau"])
        assert seed.hex() == case["seed"]
        vec = O.prf_eval_vector(seed, nonce, case["tau"], case["n"])
        exp = np.frombuffer(bytes.fromhex(case["vector"]), dtype="<u8")
        assert np.array_equal(vec, exp)


def test_lom_protect_golden(golden):
    for case in golden["lom"]["protect"]:
        nonce = bytes.fromhex(case["nonce"])
        ids = case["ids"]
        from fedbiomed_amd import workload as W

        ys = []
        for u in ids:
            x = [I(v) for v in case["x"][u]]
            y = O.lom_protect(u, W.pairwise_secrets_for(u, ids), case["tau"], x, ids, nonce)
            assert [int(v) for v in y] == [I(v) for v in case["y"][u]]
            ys.append(y)
        assert [int(v) for v in O.lom_aggregate(ys)] == [I(v) for v in case["agg"]]


def test_lom_crypter_golden(golden):
    from fedbiomed_amd import workload as W

    for case in golden["lom"]["crypter"]:
        ids = case["ids"]
        nonce = O.lom_nonce(case["nonce_str"])
        target = I(case["target"]) if case["target"] else None
        encs = []
        for u in ids:
            x = [F(v) for v in case["x"][u]]
            y = O.lom_encrypt(x, case["tau"], u, W.pairwise_secrets_for(u, ids), ids, nonce,
                              case["clip"], case["weights"][u], target)
            assert [int(v) for v in y] == [I(v) for v in case["enc"][u]]
            encs.append(y)
        agg = O.lom_crypter_aggregate(encs, case["total"], case["clip"], target)
        assert [fbits(v) for v in agg] == [s[2:] for s in case["agg"]]


def test_fdh_golden(golden):
    for case in golden["jl"]["fdh"]:
        n = I(case["n"])
        for t, h in zip(case["t"], case["h"]):
            if h == "overflow":
                with pytest.raises(OverflowError):
                    O.fdh(I(t), n * n)
            else:
                assert O.fdh(I(t), n * n) == I(h)


def test_jl_small_golden(golden):
    for case in golden["jl"]["jl_small"]:
        n = I(case["n"])
        n2 = n * n
        cts = []
        for key, ct in zip(case["keys"], case["ct"]):
            got = [((n * pt + 1) % n2) * O.powmod(O.fdh((k << 512) | case["tau"], n2), key, n2) % n2
                   for k, pt in enumerate(case["pt"])]
            assert got == [I(c) for c in ct]
            cts.append(got)
        sk0 = -sum(case["keys"])
        dec = []
        for k in range(len(case["pt"])):
            prod = math.prod(c[k] for c in cts) % n2
            v = prod * O.powmod(O.fdh((k << 512) | case["tau"], n2), sk0, n2) % n2
            dec.append(((v - 1) // n) % n)
        assert dec == [I(d) for d in case["dec"]]


@pytest.mark.parametrize("idx", range(6))
def test_jl_crypter_golden(golden, idx):
    case = golden["jl"]["crypter"][idx]
    bp = I(case["biprime"])
    target = I(case["target"]) if case["target"] else None
    P = case["n_parties"]
    encs = []
    for p in range(P):
        x = [F(v) for v in case["x"][p]]
        got = O.jl_encrypt(x, case["tau"], I(case["keys"][p]), bp, P, case["clip"], case["weights"][p], target)
        assert got == [I(c) for c in case["enc"][p]]
        encs.append(got)
    n = len(case["x"][0])
    sums = O.jl_aggregate_ints(encs, case["tau"], I(case["sk0"]), bp, n, target)
    assert sums == [I(s) for s in case["sums"]]
    bad = O.jl_aggregate_ints(encs, case["tau"], I(case["sk0"]) + 1, bp, n, target)
    assert bad == [I(s) for s in case["sums_badkey"]]
    agg = O.jl_crypter_aggregate(encs, case["tau"], I(case["sk0"]), bp, case["total"], n, case["clip"], target)
    assert [fbits(v) for v in agg] == [s[2:] for s in case["agg"]]


def test_ass_golden(golden):
    for case in golden["ass"]["cases"]:
        sh = [I(s) if isinstance(s, str) else [I(x) for x in s] for s in case["shares"]]
        rec = O.ass_reconstruct(sh)
        exp = case["reconstruct"]
        assert rec == (I(exp) if isinstance(exp, str) else [I(x) for x in exp])


def test_edge_weights_oracle(golden):
    """Negative / zero weights (tests/golden/edge.json, from the reference): the oracle's JL
    packing ORs negative products like VES._batch, and its LOM conversion raises numpy's
    OverflowError at the first negative product."""
    from fedbiomed_amd import workload as W

    edge = golden["edge"]
    for case in edge["jl"]:
        r = case["result"]
        x = [F(v) for v in case["x"]]
        if "ok" not in r or not x:
            continue
        got = O.jl_encrypt(x, case["tau"], I(case["key"]), W.BIPRIME0, case["num_nodes"], weight=case["weight"])
        assert got == [I(c) for c in r["ok"]], case["name"]
    for case in edge["lom"]:
        r = case["result"]
        x = [F(v) for v in case["x"]]
        if not x:
            continue
        ids = case["ids"]
        run = lambda: O.lom_encrypt(x, case["tau"], case["node"], W.pairwise_secrets_for(case["node"], ids),  # noqa
                                    ids, O.lom_nonce(case["nonce_str"]), weight=case["weight"])
        if "ok" in r:
            assert [int(v) for v in run()] == [I(v) for v in r["ok"]], case["name"]
        else:
            with pytest.raises(OverflowError, match=r["msg"].replace("(", r"\(").replace(")", r"\)")):
                run()
    m = edge["jl_aggregate_mixed"]
    encs = [[I(c) for c in e] for e in m["enc"]]
    keys = [I(k) for k in m["keys"]]
    agg = O.jl_crypter_aggregate(encs, m["tau"], -sum(keys), W.BIPRIME0, 2, len(m["x"]))
    assert [fbits(v) for v in agg] == [s[2:] for s in m["agg"]["ok"]]


# ---- the JoyeLibert object API fixture (tools/gen_golden.py gen_jls_api) ----
def test_jls_api_oracle(golden):
    g = golden["jls_api"]
    for case in g["fdh"]:
        m = I(case["m"])
        for t, h in zip(case["t"], case["h"]):
            if "ok" in h:
                assert O.fdh(I(t), m) == I(h["ok"])
            else:
                with pytest.raises(OverflowError):
                    O.fdh(I(t), m)
    for case in g["populate_tau"]:
        n = I(case["n"])
        if "ok" in case["h"]:
            assert [O.fdh((k << 512) | case["tau"], n * n) for k in range(case["len"])] == \
                [I(h) for h in case["h"]["ok"]]
    for case in g["user_encrypt"]:
        got = O.jl_user_encrypt([I(v) for v in case["pt"]], case["tau"], I(case["key"]), I(case["n"]))
        assert got == [I(c) for c in case["ct"]]
    for case in g["sums"]:
        n2 = I(case["n"]) ** 2
        assert math.prod(I(c) for c in case["cts"]) % n2 == I(case["sum"])
    for case in g["decrypt"]:
        n = I(case["n"])
        summed = [math.prod(col) % (n * n) for col in zip(*[[I(c) for c in row] for row in case["cts"]])]
        keys = [I(k) for k in case["keys"]]
        assert O.jl_server_decrypt(summed, case["tau"], -sum(keys), n, case["delta"]) == [I(v) for v in case["dec"]]
        assert O.jl_server_decrypt(summed, case["tau"], -sum(keys) + 1, n) == [I(v) for v in case["dec_badkey"]]
    for case, agg in zip(g["protect"], g["aggregate"]):
        n, keys = I(case["n"]), [I(k) for k in case["keys"]]
        target = I(case["target"]) if case["target"] else None
        x = [I(v) for v in case["x"]]
        for key, row in zip(keys, case["ct"]):
            assert O.jl_encrypt_ints(x, case["tau"], key, n, len(keys), target) == [I(c) for c in row]
        cts = [[I(c) for c in row] for row in case["ct"]]
        for ne, res in zip(agg["n_expected"], agg["out"]):
            assert O.jl_aggregate_ints(cts, case["tau"], -sum(keys), n, ne, target) == [I(v) for v in res["ok"]]
    for case in g["ves"]:
        es = case["valuesize"] + math.ceil(math.log2(case["add_ops"] + 1))
        cr = case["ptsize"] // es
        V = [I(v) for v in case["V"]]
        assert O.ves_encode(V, es, cr) == [I(e) for e in case["E"]]
        assert O.ves_decode([I(e) for e in case["E"]], es, cr, case["v_expected"]) == [I(v) for v in case["D"]]
