"""Seeded random cases of both crypters' list API on the HIP path against the oracle (oracle/secagg_oracle.py,
pinned to the reference's own outcomes by tests/golden/): party counts, vector lengths around the VES slot
count and the list aggregate's stripe edges, weights, clipping and target ranges, rounds up to 2^64 - 1,
keys of many lengths and both signs of the server key, num_expected_params cutting inside the vector.
Ciphertexts / masked vectors bit for bit, float64 outputs as bit patterns.  Half of the JL cases run the
list aggregate in ct_offset stripes (FBM_ONE_LANE_ROUND shrunk), some take a prepared factor, and every third
party's encrypt takes its factor computed ahead (prepare_encrypt)."""

import logging
import os
import random

import numpy as np
import pytest

from fedbiomed_amd import _device as D, workload as W

# FBM_FUZZ_CASES / FBM_FUZZ_SEED_BASE: a longer run over other seeds (round 6: profiles/r6g_fuzz_extended.txt)
N_CASES = int(os.environ.get("FBM_FUZZ_CASES", "48"))
SEED_BASE = int(os.environ.get("FBM_FUZZ_SEED_BASE", "0"))


def _bits(xs):
    return np.asarray(xs, dtype=np.float64).view(np.uint64).tolist()


def _jl_case(i):
    rng = random.Random(9100 + SEED_BASE + i)
    P = rng.randint(1, 9)
    target = rng.choice([None, 2**10, 2**16, 2**24])
    cr = D.jl_slot(target, P)[1]
    n = rng.choice([1, cr - 1, cr, cr + 1, 3 * cr, rng.randint(2, 6000), rng.randint(2, 6000)])
    clip = rng.choice([None, 1, 3, 7, 10**6])
    tau = rng.choice([0, 1, rng.getrandbits(20), 2**64 - 1])
    kbits = rng.choice([64, 700, 2040, 2040])
    keys = [rng.getrandbits(kbits) for _ in range(P)]
    weights = [rng.choice([None, 0, 1, rng.randint(1, 2**17 - 1)]) for _ in range(P)]
    scale = (clip or 3) * rng.choice([0.3, 1.0, 1.7])
    x = [[rng.uniform(-scale, scale) for _ in range(n)] for _ in range(P)]
    n_exp = rng.choice([n, max(1, n // 2), n + 5])
    sign = rng.choice([-1, -1, -1, 1])  # the reference's server key is -sum(keys); + takes the factor's other path
    return dict(P=P, n=n, cr=cr, target=target, clip=clip, tau=tau, keys=keys, weights=weights, x=x, n_exp=n_exp,
                sign=sign, striped=i % 2 == 1, prepared=i % 3 == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(N_CASES))
def test_jl_fuzz_vs_oracle(i, monkeypatch, caplog):
    from oracle import secagg_oracle as O
    from fedbiomed_amd.secagg import SecaggCrypter

    caplog.set_level(logging.ERROR)
    c = _jl_case(i)
    jc = SecaggCrypter()
    cts = []
    for p in range(c["P"]):
        if (i + p) % 3 == 0:  # some parties' encrypts with their factor computed ahead (prepare_encrypt)
            assert jc.prepare_encrypt(c["tau"], c["P"], c["keys"][p], W.BIPRIME0, c["n"], target_range=c["target"])
        got = jc.encrypt(c["P"], c["tau"], c["x"][p], c["keys"][p], W.BIPRIME0, clipping_range=c["clip"],
                         weight=c["weights"][p], target_range=c["target"])
        ref = O.jl_encrypt(c["x"][p], c["tau"], c["keys"][p], W.BIPRIME0, c["P"], clip=c["clip"],
                           weight=c["weights"][p], target=c["target"])
        assert got == ref, (i, p)
        cts.append(got)
    total = sum(w if w is not None else 1 for w in c["weights"]) or 1
    sk0 = c["sign"] * sum(c["keys"])
    ref = O.jl_crypter_aggregate(cts, c["tau"], sk0, W.BIPRIME0, total, c["n_exp"], clip=c["clip"],
                                 target=c["target"])
    if c["striped"]:
        monkeypatch.setenv("FBM_ONE_LANE_ROUND", str(max(1, len(cts[0]) // 3)))
    if c["prepared"]:
        assert jc.prepare_aggregate(c["tau"], c["P"], sk0, W.BIPRIME0, c["n_exp"], target_range=c["target"])
    out = jc.aggregate(c["tau"], c["P"], cts, sk0, W.BIPRIME0, total, clipping_range=c["clip"],
                       num_expected_params=c["n_exp"], target_range=c["target"])
    assert _bits(out) == _bits(ref), i


def _lom_case(i):
    rng = random.Random(9300 + SEED_BASE + i)
    P = rng.randint(2, 12)
    n = rng.choice([1, 7, 8, 9, rng.randint(2, 6000)])
    target = rng.choice([None, 2**10, 2**20])
    clip = rng.choice([None, 1, 3, 10**3])
    tau = rng.choice([0, rng.getrandbits(30), 2**40 + 7])
    weights = [rng.choice([None, 1, rng.randint(1, 2**17 - 1)]) for _ in range(P)]
    scale = (clip or 3) * rng.choice([0.5, 1.4])
    x = [[rng.uniform(-scale, scale) for _ in range(n)] for _ in range(P)]
    return dict(P=P, n=n, target=target, clip=clip, tau=tau, weights=weights, x=x,
                nonce=rng.choice([None, "secagg_fuzz_%d" % i]))


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(N_CASES))
def test_lom_fuzz_vs_oracle(i, caplog):
    from oracle import secagg_oracle as O
    from fedbiomed_amd.secagg import SecaggLomCrypter

    caplog.set_level(logging.ERROR)
    c = _lom_case(i)
    ids = W.node_ids(c["P"])
    lc = SecaggLomCrypter(c["nonce"] or "secagg_default")
    nonce = O.lom_nonce(c["nonce"] or "secagg_default")
    ys = []
    for p, u in enumerate(ids):
        sec = W.pairwise_secrets_for(u, ids)
        if (i + p) % 2 == 0:  # the output's ints made ahead (prepare_encrypt)
            lc.prepare_encrypt(c["tau"], u, c["n"])
        got = lc.encrypt(c["tau"], u, c["x"][p], sec, ids, clipping_range=c["clip"], weight=c["weights"][p],
                         target_range=c["target"])
        ref = O.lom_encrypt(np.asarray(c["x"][p], np.float64), c["tau"], u, sec, ids, nonce, clip=c["clip"],
                            weight=c["weights"][p], target=c["target"])
        assert got == [int(v) for v in np.asarray(ref, dtype=np.uint64)], (i, p)
        ys.append(got)
    total = sum(w if w is not None else 1 for w in c["weights"])
    if i % 2:  # the output's floats made ahead (prepare_aggregate)
        assert lc.prepare_aggregate(c["n"])
    out = lc.aggregate(ys, total, clipping_range=c["clip"], target_range=c["target"])
    ref = O.lom_crypter_aggregate([np.asarray(y, dtype=np.uint64) for y in ys], total, clip=c["clip"],
                                  target=c["target"])
    assert _bits(out) == _bits(ref), i
