"""Both crypters over a broad sweep of the reference's own outcomes (tests/golden/crypter_sweep.json,
tools/gen_golden.py gen_crypter_sweep): party counts 1..17, ragged lengths around the VES slot
counts, rounds 0 and 2^64 - 1, unweighted / weighted (incl. the largest weight), clipping ranges
1 .. 1e14, target ranges 7 .. 2^64, clipped values, exact halves, signed zeros -- ciphertexts /
masked vectors and float64 outputs bit for bit, errors by type and message.  The oracle is checked
against the same outcomes on the CPU; the crypters run the HIP path."""

import logging

import numpy as np
import pytest

from fedbiomed_amd import workload as W
from tests.golden_util import F, I


def _run(outcome, fn):
    """Compare fn() with a golden {"ok": ...} / {"error": type, "msg": ...} outcome; returns fn()'s
    value (None on an expected error)."""
    if "error" in outcome:
        with pytest.raises(Exception) as ei:
            fn()
        assert type(ei.value).__name__ == outcome["error"]
        assert str(ei.value) == outcome["msg"]
        return None
    return fn()


def _bits(xs):
    return np.asarray(xs, dtype=np.float64).view(np.uint64).tolist()


def _case_ids(kind):
    from tests.golden_util import load

    return [f"{kind}{i}-P{c['P']}-n{c['n']}" for i, c in enumerate(load("crypter_sweep.json")[kind])]


@pytest.mark.parametrize("idx", range(len(_case_ids("jl"))), ids=_case_ids("jl"))
def test_jl_sweep_oracle(golden, idx):
    from oracle import secagg_oracle as O

    c = golden["crypter_sweep"]["jl"][idx]
    target = I(c["target"]) if c["target"] else None
    keys = [I(k) for k in c["keys"]]
    for p, e in enumerate(c["enc"]):
        got = _run(e, lambda p=p: O.jl_encrypt([F(v) for v in c["x"][p]], c["tau"], keys[p], W.BIPRIME0, c["P"],
                                               clip=c["clip"], weight=c["weights"][p], target=target))
        if got is None:  # an expected error: the reference skipped the aggregate
            return
        assert got == [I(v) for v in e["ok"]]
    cts = [[I(v) for v in e["ok"]] for e in c["enc"]]
    out = O.jl_crypter_aggregate(cts, c["tau"], -sum(keys), W.BIPRIME0, c["total"], c["n"], clip=c["clip"],
                                 target=target)
    assert _bits(out) == _bits([F(v) for v in c["agg"]["ok"]])


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(len(_case_ids("jl"))), ids=_case_ids("jl"))
def test_jl_sweep_gpu(golden, idx, caplog):
    from fedbiomed_amd.secagg import SecaggCrypter

    c = golden["crypter_sweep"]["jl"][idx]
    target = I(c["target"]) if c["target"] else None
    keys = [I(k) for k in c["keys"]]
    jc = SecaggCrypter()
    with caplog.at_level(logging.WARNING):
        encs = [_run(e, lambda p=p: jc.encrypt(num_nodes=c["P"], current_round=c["tau"], params=[F(v) for v in c["x"][p]],
                                               key=keys[p], biprime=W.BIPRIME0, clipping_range=c["clip"],
                                               weight=c["weights"][p], target_range=target))
                for p, e in enumerate(c["enc"])]
    for got, e in zip(encs, c["enc"]):
        assert got == ([I(v) for v in e["ok"]] if "ok" in e else None)
    if c["agg"].get("error") == "skipped":  # an encrypt failed (as expected): nothing to aggregate
        return
    out = _run(c["agg"], lambda: jc.aggregate(current_round=c["tau"], num_nodes=c["P"], params=encs, key=-sum(keys),
                                              biprime=W.BIPRIME0, total_sample_size=c["total"],
                                              clipping_range=c["clip"], num_expected_params=c["n"],
                                              target_range=target))
    if out is not None:
        assert _bits(out) == _bits([F(v) for v in c["agg"]["ok"]])


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(len(_case_ids("lom"))), ids=_case_ids("lom"))
def test_lom_sweep_gpu(golden, idx, caplog):
    from fedbiomed_amd.secagg import SecaggLomCrypter

    c = golden["crypter_sweep"]["lom"][idx]
    target = I(c["target"]) if c["target"] else None
    ids = c["ids"]
    encs = []
    with caplog.at_level(logging.WARNING):
        for p, e in enumerate(c["enc"]):
            got = _run(e, lambda p=p: SecaggLomCrypter(nonce=c["nonce_str"]).encrypt(
                current_round=c["tau"], node_id=ids[p], params=[F(v) for v in c["x"][p]],
                pairwise_secrets=W.pairwise_secrets_for(ids[p], ids), node_ids=ids, clipping_range=c["clip"],
                weight=c["weights"][p], target_range=target))
            if got is not None:
                assert got == [I(v) for v in e["ok"]]
            encs.append(got)
    if "ok" in c["agg"]:
        out = SecaggLomCrypter(nonce=c["nonce_str"]).aggregate(encs, c["total"], clipping_range=c["clip"],
                                                               target_range=target)
        assert _bits(out) == _bits([F(v) for v in c["agg"]["ok"]])


@pytest.mark.parametrize("idx", range(len(_case_ids("lom"))), ids=_case_ids("lom"))
def test_lom_sweep_oracle(golden, idx):
    from oracle import secagg_oracle as O

    c = golden["crypter_sweep"]["lom"][idx]
    target = I(c["target"]) if c["target"] else None
    ids, nonce = c["ids"], O.lom_nonce(c["nonce_str"])
    encs = []
    for p, e in enumerate(c["enc"]):
        try:
            got = O.lom_encrypt([F(v) for v in c["x"][p]], c["tau"], ids[p], W.pairwise_secrets_for(ids[p], ids), ids,
                                nonce, clip=c["clip"], weight=c["weights"][p], target=target)
        except (O.OracleError, OverflowError) as err:
            assert "error" in e
            if isinstance(err, OverflowError):
                assert (type(err).__name__, str(err)) == (e["error"], e["msg"])
            else:
                assert e["error"] == "FedbiomedSecaggError" and str(err)[:6] == e["msg"][:6]
            encs.append(None)
            continue
        assert [int(v) for v in got] == [I(v) for v in e["ok"]]
        encs.append(got)
    if "ok" in c["agg"]:
        out = O.lom_crypter_aggregate(encs, c["total"], clip=c["clip"], target=target)
        assert _bits(out) == _bits([F(v) for v in c["agg"]["ok"]])


@pytest.mark.gpu
def test_lom_round_counter_edges():
    """PRF.eval_vector's (i + tau).to_bytes(8, 'big') (_lom.py:81) at the top of the round counter:
    the last tau that fits is bit-exact with the oracle, one more is the reference's OverflowError
    -- after its overflow guard (FB417 wins), and never without peers."""
    from oracle import secagg_oracle as O
    from fedbiomed_amd.exceptions import FedbiomedSecaggError
    from fedbiomed_amd.secagg import LOM

    ids, nonce = ["a", "b", "c"], bytes(range(16))
    sec = W.pairwise_secrets_for("b", ids)
    x = list(range(1, 20))
    top = 2 ** 64 - len(x)
    y = LOM(nonce=nonce).protect("b", sec, top, x, ids)
    assert y == [int(v) for v in O.lom_protect("b", sec, top, x, ids, nonce)]
    for tau, msg in ((top + 1, "int too big to convert"), (2 ** 64 + 3, "int too big to convert"),
                     (-1, "can't convert negative int to unsigned")):
        with pytest.raises(OverflowError, match=msg):
            LOM(nonce=nonce).protect("b", sec, tau, x, ids)
        with pytest.raises(OverflowError, match=msg):
            O.lom_protect("b", sec, tau, x, ids, nonce)
        with pytest.raises(FedbiomedSecaggError):  # the overflow guard first
            LOM(nonce=nonce).protect("b", sec, tau, [2 ** 62] + x, ids)
    assert LOM(nonce=nonce).protect("b", {}, top + 1, x, ["b"]) == x  # no peers: no PRF call


def test_lom_overflow_message_word_for_word(golden):
    """The overflow guard's message (secagg/_lom.py:137-149) as the host mirror builds it from the
    status words, against the reference's own text in the sweep fixture (CPU: no device call)."""
    import re

    from fedbiomed_amd import _device as D

    seen = 0
    for c in golden["crypter_sweep"]["lom"]:
        for e in c["enc"]:
            if e.get("error") == "FedbiomedSecaggError" and "overflow detected" in e["msg"]:
                bits = int(re.search(r"requires (\d+) bits", e["msg"]).group(1))
                assert D._lom_overflow_message(bits, c["P"]) == e["msg"]
                seen += 1
    assert seen
