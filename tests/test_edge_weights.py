"""Weight edge cases of the drop-in crypters against the reference's own outcomes
(tests/golden/edge.json, written by tools/gen_golden.py from /root/reference).

Reference behaviour (`_secagg_crypter.py:45-137,318-392`):
* the weight bound (2**w.bit_length() <= 2^17) is checked after quantize and before the
  scheme's protect, so an empty `params` with a too-large weight raises FB624, while an empty
  JL encrypt otherwise returns [] and an empty LOM encrypt raises FB624 "max() arg ...";
* a negative weight passes that bound: JL encrypts the OR-packed negative products
  (VES._batch, `_jls.py:169-176`), LOM raises numpy's OverflowError at the first negative
  product (`_lom.py:153`), unless every product is 0.

The ordering cases need no device (they raise or return before any kernel); the compute
cases run the HIP path (`-m gpu`) and compare bit for bit.
"""

import pytest

from fedbiomed_amd import workload as W
from tests.golden_util import F, I, fbits


def _jl(case):
    from fedbiomed_amd.secagg import SecaggCrypter

    return SecaggCrypter().encrypt(num_nodes=case["num_nodes"], current_round=case["tau"],
                                   params=[F(v) for v in case["x"]], key=I(case["key"]), biprime=W.BIPRIME0,
                                   weight=case["weight"])


def _lom(case):
    from fedbiomed_amd.secagg import SecaggLomCrypter

    ids = case["ids"]
    return SecaggLomCrypter(nonce=case["nonce_str"]).encrypt(
        current_round=case["tau"], node_id=case["node"], params=[F(v) for v in case["x"]],
        pairwise_secrets=W.pairwise_secrets_for(case["node"], ids), node_ids=ids, weight=case["weight"])


def _check(run, case):
    r = case["result"]
    if "ok" in r:
        assert [hex(int(v)) for v in run(case)] == r["ok"], case["name"]
        return
    with pytest.raises(Exception) as ei:
        run(case)
    assert type(ei.value).__name__ == r["error"], case["name"]
    assert str(ei.value) == r["msg"], case["name"]


def _cases(golden, scheme, device):
    out = []
    for c in golden["edge"][scheme]:
        host_only = not c["x"] or "big" in c["name"]  # raises / returns before any kernel
        if host_only != device:
            out.append(c)
    return out


def test_edge_order_host(golden):
    """Empty inputs and too-large weights: same outcome as the reference, no device needed."""
    cases = _cases(golden, "jl", False) + _cases(golden, "lom", False)
    assert len(cases) >= 5
    for c in _cases(golden, "jl", False):
        _check(_jl, c)
    for c in _cases(golden, "lom", False):
        _check(_lom, c)


@pytest.mark.gpu
def test_edge_negative_weights_jl_gpu(golden):
    cases = _cases(golden, "jl", True)
    assert {c["name"] for c in cases} >= {"neg3", "neg1", "neg_max", "w0", "neg_lowfirst", "neg_allzero"}
    for c in cases:
        _check(_jl, c)


@pytest.mark.gpu
def test_edge_negative_weights_lom_gpu(golden):
    cases = _cases(golden, "lom", True)
    assert {c["name"] for c in cases} >= {"neg3", "neg_lowfirst", "neg_allzero", "w0"}
    for c in cases:
        _check(_lom, c)


@pytest.mark.gpu
def test_edge_mixed_sign_aggregate_gpu(golden):
    from fedbiomed_amd.secagg import SecaggCrypter

    m = golden["edge"]["jl_aggregate_mixed"]
    keys = [I(k) for k in m["keys"]]
    x = [F(v) for v in m["x"]]
    enc = [SecaggCrypter().encrypt(2, m["tau"], x, keys[p], W.BIPRIME0, weight=w) for p, w in enumerate(m["weights"])]
    assert enc == [[I(c) for c in e] for e in m["enc"]]
    agg = SecaggCrypter().aggregate(m["tau"], 2, enc, -sum(keys), W.BIPRIME0, 2, num_expected_params=len(x))
    assert [fbits(v) for v in agg] == [s[2:] for s in m["agg"]["ok"]]
