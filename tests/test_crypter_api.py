"""The reference's own crypter and utility test flows (tests/test_secagg_crypter.py:118-381,
tests/test_secagg_utils.py:51-120), restated for the mirror: target-range forwarding, encrypt /
aggregate argument validation, the decrypt round trip, the federated-analytics wide-range round
trip and the quantise / weight / average identities.  The crypters and quantize / reverse_quantize
run the HIP kernels (GPU tests); multiply / divide are host integer helpers (CPU)."""

import copy
from math import ceil, log2

import pytest

from fedbiomed_amd.constants import SAParameters
from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError
from fedbiomed_amd.utils import divide, multiply, quantize, reverse_quantize

# the reference test's biprime (test_secagg_crypter.py:14)
BIPRIME = int(
    "158820908809271716671659880613366104677813341255487834154303909761107215283569995523817428402987962641429"
    "395032343305343341950966867458277812575065022203120547706127493272939455658018882112230042773163870472621"
    "818892994896895819790062496734944602899772583591514631486212290112369502692304700112819186167541107")

WEIGHTS = (
    [[0.1, 0.2, 0.3], [0.4, 0.5, 0.6], [0.7, 0.8, 0.9]],
    [[0.1], [0.2], [0.3]],
    [[0.1, 0.2, 0.3]],
    [[0.1, 0.2, 0.3], [0.4, 0.5, 0.6], [0.7, 0.8, 0.9], [0.1, 0.11, 0.12], [0.1, 0.13, 0.14]],
)
MULTIPLIERS = ([1, 2, 3], [1, 2, 3], [2], [5, 4, 3, 2, 1])


def _quantize_and_aggregate(weights, n_nodes, clip, target, multipliers=None):
    """test_secagg_utils.py:27-49"""
    weights = copy.deepcopy(weights)
    q = [quantize(w, clip, target) for w in weights]
    if multipliers is not None:
        for i in range(n_nodes):
            q[i] = multiply(q[i], multipliers[i])
            weights[i] = multiply(weights[i], multipliers[i])
    sum_q = [sum(w) for w in zip(*q)]
    sum_w = [sum(w) for w in zip(*weights)]
    divisor = sum(multipliers) if multipliers else n_nodes
    return divide(sum_w, divisor), reverse_quantize(divide(sum_q, divisor), clip, target)


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True], ids=["unweighted", "weighted"])
def test_utils_average_of_quantized(weighted):
    """test_secagg_utils.py:51-75: reverse_quantize(divide(multiply(quantize(w)))) ~ divide(multiply(w))"""
    for weights, mult in zip(WEIGHTS, MULTIPLIERS):
        plain, restored = _quantize_and_aggregate(weights, len(weights), 2, 2 ** 16, mult if weighted else None)
        for a, b in zip(plain, restored):
            assert a == pytest.approx(b, abs=5e-4)


def test_utils_multiply_divide():
    """test_secagg_utils.py:77-120"""
    weights_collection = (
        [[0.1, 0.2, 0.3], [0.4, 0.5, 0.6], [0.7, 0.8, 0.9]],
        [[0.11, 0.21, 0.54]],
        [[0.1], [0.2], [0.3]],
        [[0.1, 0.5, 77], [0.5, 0.67, 0.44, 0.55, 0.02], [0.2, 0.4], [0.1, 0.1, 0.1, 0.0]],
    )
    for weights, mult in zip(weights_collection, ([1, 2, 3], [3], [1, 2, 3], [1, 2, 3])):
        back = [divide(multiply(w, k), k) for w, k in zip(weights, mult)]
        for w1, w2 in zip(weights, back):
            assert w2 == pytest.approx(w1, abs=1e-5)


@pytest.mark.gpu
def test_crypter_target_range_forwarding():
    """test_secagg_crypter.py:118-166: encrypt / aggregate take target_range (None -> TARGET_RANGE)"""
    from fedbiomed_amd.secagg import SecaggCrypter

    sc = SecaggCrypter()
    params = [1.0, 2.0, 3.0, 4.0]
    enc = dict(num_nodes=2, current_round=1, params=params, biprime=BIPRIME, key=10)
    assert sc.encrypt(**enc) == sc.encrypt(**enc, target_range=SAParameters.TARGET_RANGE)
    assert sc.encrypt(**enc) != sc.encrypt(**enc, target_range=SAParameters.FA_TARGET_RANGE)
    e = [sc.encrypt(num_nodes=2, current_round=2, params=[0.5, 0.8], biprime=BIPRIME, key=10,
                    target_range=SAParameters.FA_TARGET_RANGE) for _ in range(2)]
    agg = dict(current_round=2, num_nodes=2, params=e, biprime=BIPRIME, key=-20, total_sample_size=2,
               num_expected_params=2)
    fa = sc.aggregate(**agg, target_range=SAParameters.FA_TARGET_RANGE)
    assert fa == pytest.approx([0.5, 0.8], abs=1e-9)
    assert sc.aggregate(**agg) != fa  # the default range decodes the FA-range sums differently


@pytest.mark.gpu
def test_crypter_encrypt_validation():
    """test_secagg_crypter.py:168-228"""
    from fedbiomed_amd.secagg import SecaggCrypter

    sc = SecaggCrypter()
    kw = dict(num_nodes=2, current_round=1, biprime=BIPRIME, key=10)
    result = sc.encrypt(params=[10.0, 20.0, 30.0, 40.0], **kw)
    assert isinstance(result, list)
    assert ceil(log2(int(result[0]))) <= BIPRIME.bit_length() * 2
    for bad in ("not-a-list", ["not-a-float", "not-a-float"], [0, 1, 2]):
        with pytest.raises(FedbiomedSecaggCrypterError):
            sc.encrypt(params=bad, **kw)
    with pytest.raises(FedbiomedSecaggCrypterError):  # the key must be an integer
        sc.encrypt(params=[1.0], num_nodes=2, current_round=1, biprime=BIPRIME, key=10.0)


@pytest.mark.gpu
def test_crypter_decrypt_round_trip_and_validation():
    """test_secagg_crypter.py:230-326"""
    from fedbiomed_amd.secagg import SecaggCrypter

    sc = SecaggCrypter()
    params = [0.5, 0.8, -0.5, 0.0]
    nodes = [sc.encrypt(num_nodes=2, current_round=2, params=params, biprime=BIPRIME, key=10) for _ in range(2)]
    agg = dict(current_round=2, num_nodes=2, key=-20, biprime=BIPRIME, total_sample_size=8)
    result = sc.aggregate(params=nodes, num_expected_params=len(params), **agg)
    assert len(result) == len(params)
    # the summed quantised values averaged over total_sample_size 8, then dequantised
    expected = reverse_quantize(divide([2 * q for q in quantize(params)], 8))
    assert result == expected
    for bad in ([[1, 1, 1], [2, 2, 2], [3, 3, 3]],  # three parties for num_nodes = 2
                [["not-int"] * 3, ["not-int"] * 3],  # not integers
                ["not-int", "not-int"]):  # not a list of lists
        with pytest.raises(FedbiomedSecaggCrypterError):
            sc.aggregate(params=bad, **agg)


@pytest.mark.gpu
def test_crypter_fa_wide_range_round_trip():
    """test_secagg_crypter.py:328-377: ~55-bit federated-analytics statistics in adjacent slots"""
    from fedbiomed_amd.secagg import SecaggCrypter

    sc = SecaggCrypter()
    C, T = SAParameters.FA_CLIPPING_RANGE, SAParameters.FA_TARGET_RANGE
    enc = [sc.encrypt(num_nodes=2, current_round=1, params=v, key=10, biprime=BIPRIME, clipping_range=C, weight=1,
                      target_range=T) for v in ([10667.0, 21516413.0], [17965.0, 36233008.0])]
    out = sc.aggregate(current_round=1, num_nodes=2, params=enc, key=-20, biprime=BIPRIME, total_sample_size=2,
                       clipping_range=C, num_expected_params=2, target_range=T)
    assert [v * 2 for v in out] == pytest.approx([28632.0, 57749421.0], abs=1.0)


@pytest.mark.gpu
def test_list_encrypt_overlapped_stripes_equal_unsplit(monkeypatch, caplog):
    """the list API's encrypt runs as ct_offset stripes (full one-lane rounds, the
    partial round last) with each stripe's Python ints built while the next stripe exponentiates.
    The returned list is bit-identical to the unsplit call's, errors and the clipping warning (once)
    are as before.  FBM_ONE_LANE_ROUND shrinks the round so small vectors split."""
    import logging

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    P, tau, n = 4, 3, 40_003
    xs = [float(v) for v in W.party_params(2, n)]
    key = W.jl_user_key(2)
    jc = SecaggCrypter()
    ref = jc.encrypt(P, tau, xs, key, W.BIPRIME0, weight=7)
    for rnd in ("300", "431", "645"):  # 645: a 1-ciphertext sliver rides with the last round
        monkeypatch.setenv("FBM_ONE_LANE_ROUND", rnd)
        _, cr = D.jl_slot(None, P)
        stripes = D.list_encrypt_stripes((n + cr - 1) // cr)
        assert len(stripes) > 1 and stripes[0] == (0, int(rnd)) and stripes[-1][1] == (n + cr - 1) // cr
        caplog.clear()
        with caplog.at_level(logging.WARNING, logger="fedbiomed_amd"):
            got = jc.encrypt(P, tau, xs, key, W.BIPRIME0, weight=7)
        assert got == ref
        assert sum("exceeds clipping range" in r.getMessage() for r in caplog.records) == 1
    monkeypatch.setenv("FBM_ONE_LANE_ROUND", "300")
    with pytest.raises(Exception):
        jc.encrypt(P, tau, xs[:-1] + [1], key, W.BIPRIME0)  # a non-float: FB624 before any device work


@pytest.mark.gpu
def test_list_aggregate_stripes_equal_unsplit(monkeypatch):
    """Round 5: the researcher's aggregate(List[List[int]]) runs as ct_offset stripes (stripe k's combine and
    D2H, then stripe k + 1's factor; stripe k + 1's ints converted in the background while stripe k's floats are
    written in place).  Bit-identical to the unsplit call for
    every stripe plan, with num_expected_params cutting inside a stripe, at a stripe edge, past the end and at
    0, ragged lists (zip truncation), out-of-range ciphertexts in any stripe and the wire blob; errors as before
    (a zero sample size, a bad item)."""
    from fedbiomed_amd import _device as D, wire, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    P, tau, n = 4, 5, 30_001
    keys = [W.jl_user_key(p) for p in range(P)]
    jc = SecaggCrypter()
    cl = [jc.encrypt(P, tau, [float(v) for v in W.party_params(p, n)], keys[p], W.BIPRIME0, weight=3 + p)
          for p in range(P)]
    cl[1] = cl[1] + [12345]  # ragged: zip truncates
    tw = sum(3 + p for p in range(P))
    _, cr = D.jl_slot(None, P)
    monkeypatch.delenv("FBM_ONE_LANE_ROUND", raising=False)
    cases = [n, 7, 250 * cr, 250 * cr + 1, n + 100, 0]
    ref = {e: jc.aggregate(tau, P, cl, -sum(keys), W.BIPRIME0, tw, num_expected_params=e) for e in cases}
    assert len(D.list_encrypt_stripes(len(cl[0]))) == 1
    for rnd in ("250", "333"):
        monkeypatch.setenv("FBM_ONE_LANE_ROUND", rnd)
        assert len(D.list_encrypt_stripes(len(cl[0]))) > 2
        for e in cases:
            assert jc.aggregate(tau, P, cl, -sum(keys), W.BIPRIME0, tw, num_expected_params=e) == ref[e], (rnd, e)
        with pytest.raises(ZeroDivisionError):
            jc.aggregate(tau, P, cl, -sum(keys), W.BIPRIME0, 0, num_expected_params=n)
        bad = [list(c) for c in cl]
        bad[2][5] = 1.5
        with pytest.raises(Exception, match="FB624"):
            jc.aggregate(tau, P, bad, -sum(keys), W.BIPRIME0, tw, num_expected_params=n)
        # values outside [0, N^2) in a later stripe: the background conversion's slow path reduces them
        n2 = W.BIPRIME0 ** 2
        shifted = [list(c) for c in cl]
        shifted[3][600] += n2
        shifted[0][700] -= n2
        shifted[1][2] += 5 * n2  # stripe 0 too
        assert jc.aggregate(tau, P, shifted, -sum(keys), W.BIPRIME0, tw, num_expected_params=n) == ref[n], rnd
    monkeypatch.setenv("FBM_ONE_LANE_ROUND", "250")
    wire.enable()
    try:
        cw = [jc.encrypt(P, tau, [float(v) for v in W.party_params(p, n)], keys[p], W.BIPRIME0, weight=3 + p)
              for p in range(P)]
        assert jc.aggregate(tau, P, cw, -sum(keys), W.BIPRIME0, tw, num_expected_params=n) == ref[n]
    finally:
        wire.enable(False)


@pytest.mark.gpu
def test_prepare_aggregate_factor_ahead(monkeypatch):
    """prepare_aggregate (an extension): the decryption factor issued before the parties' lists exist.  The
    next aggregate of the same round / key / biprime / node count / size takes it and is bit-identical to an
    unprepared call, striped or not; it is used once; another call of the round leaves it (the researcher's
    validation aggregate comes first), a call of another round drops it; arguments aggregate would refuse
    prepare nothing."""
    from fedbiomed_amd import workload as W
    from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter

    P, tau, n = 4, 6, 20_011
    keys = [W.jl_user_key(p) for p in range(P)]
    sk0 = -sum(keys)
    jc = SecaggCrypter()
    cl = [jc.encrypt(P, tau, [float(v) for v in W.party_params(p, n)], keys[p], W.BIPRIME0, weight=2 + p)
          for p in range(P)]
    tw = sum(2 + p for p in range(P))
    for rnd in (None, "200"):
        if rnd is None:
            monkeypatch.delenv("FBM_ONE_LANE_ROUND", raising=False)
        else:
            monkeypatch.setenv("FBM_ONE_LANE_ROUND", rnd)
        ref = jc.aggregate(tau, P, cl, sk0, W.BIPRIME0, tw, num_expected_params=n)
        assert jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n) is True
        assert jc._prepared is not None
        assert jc.aggregate(tau, P, cl, sk0, W.BIPRIME0, tw, num_expected_params=n) == ref, rnd
        assert jc._prepared is None  # spent
        assert jc.aggregate(tau, P, cl, sk0, W.BIPRIME0, tw, num_expected_params=n) == ref
        # another round's preparation is dropped by this round's call
        assert jc.prepare_aggregate(tau + 1, P, sk0, W.BIPRIME0, n) is True
        assert jc.aggregate(tau, P, cl, sk0, W.BIPRIME0, tw, num_expected_params=n) == ref
        assert jc._prepared is None
        # same round, another key / size: ignored and kept
        for other in ((tau, P, sk0 - 1, W.BIPRIME0, n), (tau, P, sk0, W.BIPRIME0, n + 10_000)):
            assert jc.prepare_aggregate(*other) is True
            assert jc.aggregate(tau, P, cl, sk0, W.BIPRIME0, tw, num_expected_params=n) == ref, other
            assert jc._prepared is not None
        # the researcher's flow (_secure_aggregation.py:354-401): the insecure-validation aggregate of
        # one-ciphertext encryption factors first, then the model's -- which takes the preparation
        ef = [jc.encrypt(P, tau, [0.25], keys[p], W.BIPRIME0, weight=2 + p) for p in range(P)]
        val_ref = jc.aggregate(tau, P, ef, sk0, W.BIPRIME0, tw, num_expected_params=1)
        assert jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n) is True
        assert jc.aggregate(tau, P, ef, sk0, W.BIPRIME0, tw, num_expected_params=1) == val_ref
        assert jc._prepared is not None
        assert jc.aggregate(tau, P, cl, sk0, W.BIPRIME0, tw, num_expected_params=n) == ref
        assert jc._prepared is None
    # the wire blobs' packed rows (no int conversion) take the prepared factor too
    from fedbiomed_amd import wire

    monkeypatch.setenv("FBM_ONE_LANE_ROUND", "200")
    wire.enable()
    try:
        cw = [jc.encrypt(P, tau, [float(v) for v in W.party_params(p, n)], keys[p], W.BIPRIME0, weight=2 + p)
              for p in range(P)]
        assert jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n) is True
        assert jc.aggregate(tau, P, cw, sk0, W.BIPRIME0, tw, num_expected_params=n) == ref
        assert jc._prepared is None
    finally:
        wire.enable(False)
    for bad in ((tau, P, 1.5, W.BIPRIME0, n), (tau, P, sk0, W.BIPRIME0, 0), (tau, 0, sk0, W.BIPRIME0, n),
                (tau, P, sk0, "N", n)):
        assert jc.prepare_aggregate(*bad) is False
    assert SecaggLomCrypter().prepare_aggregate(tau, P, sk0, W.BIPRIME0, n) is False
