"""Concurrent callers and key-material hygiene.

The reference is single-threaded per call, but a node runs its encrypt on its task thread
(fedbiomed/node/node.py:569-630) while other threads may be running, and the researcher
aggregates on its main thread.  The library's per-thread state (the engine / short-path policy of
the test build, the exponentiation batch, the last error) must keep two threads' calls apart:
  * a JL encrypt on one thread and a LOM aggregate on another, at once, equal the serial calls;
  * one thread pinned to the triple engine (test build) and another on the product library's
    policy, at once, both bit-equal to the serial results -- the switch does not leak.
Hygiene: the node's prepared H(t_k)^key factor is zeroed and dropped by drop_prepared, by the
clear-caches path and by an encrypt that raises; the synchronous host calls' device workspace is
zeroed behind each call and released by the clear-caches path.
"""

import threading

import numpy as np
import pytest
import torch

from fedbiomed_amd import _device as D, workload as W

pytestmark = pytest.mark.gpu


def _run_threads(*fns):
    """Runs each fn on its own thread and its own HIP stream, all released at once; returns their results."""
    dev = D.device()
    gate = threading.Barrier(len(fns))
    out, errs = [None] * len(fns), []

    def body(i, fn):
        try:
            s = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(s):
                gate.wait(timeout=60)
                r = fn()
                s.synchronize()
            out[i] = r
        except BaseException as e:  # noqa: BLE001 -- surfaced below
            errs.append(e)

    ts = [threading.Thread(target=body, args=(i, f)) for i, f in enumerate(fns)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    if errs:
        raise errs[0]
    return out


def test_jl_encrypt_and_lom_aggregate_on_two_threads():
    from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter

    dev = D.device()
    P, tau, n = 4, 3, 50_000
    ids, ws = W.node_ids(P), [W.party_weight(p) for p in range(P)]
    keys = [W.jl_user_key(p) for p in range(P)]
    xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
    jc, lc = SecaggCrypter(), SecaggLomCrypter(W.LOM_NONCE)
    Y = torch.stack([lc.encrypt_tensor(tau, u, xs[p], W.pairwise_secrets_for(u, ids), ids, weight=ws[p])
                     for p, u in enumerate(ids)])

    def jl():
        return torch.stack([jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p])
                            for p in range(P)]).cpu()

    def lom():
        return lc.aggregate_tensor(Y, sum(ws)).cpu()

    ref_jl, ref_lom = jl(), lom()
    for _ in range(3):
        got_jl, got_lom = _run_threads(jl, lom)
        assert torch.equal(got_jl, ref_jl) and torch.equal(got_lom, ref_lom)
    # and the list API: one node's encrypt beside the researcher's LOM aggregate
    xl = W.party_params(0, 3_000).astype(np.float64).tolist()
    yl = [lc.encrypt(tau, u, W.party_params(p, 3_000).astype(np.float64).tolist(), W.pairwise_secrets_for(u, ids),
                     ids, weight=ws[p]) for p, u in enumerate(ids)]
    ref = (jc.encrypt(P, tau, xl, keys[0], W.BIPRIME0, weight=ws[0]), lc.aggregate(yl, sum(ws)))
    got = _run_threads(lambda: jc.encrypt(P, tau, xl, keys[0], W.BIPRIME0, weight=ws[0]),
                       lambda: lc.aggregate(yl, sum(ws)))
    assert got[0] == ref[0] and np.asarray(got[1]).view(np.uint64).tolist() == np.asarray(ref[1]).view(
        np.uint64).tolist()


def test_engine_switch_is_per_thread():
    """Thread A encrypts under the test build's triple engine, thread B through the product library at
    the same time: both equal the serial results, and B's launch took the product's own policy."""
    from fedbiomed_amd import _native
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau, n = 3, 7, 30_000
    keys = [W.jl_user_key(p) for p in range(P)]
    xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
    jc = SecaggCrypter()

    def enc():
        return torch.stack([jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0) for p in range(P)]).cpu()

    ref = enc()
    seen = {}

    def pinned():
        with D.jl_engine("triple"):
            seen["a"] = D.jl_engine_for(10**7)
            return enc()

    def plain():
        seen["b_lib_is_product"] = _native.load() is not _native.load_test()
        return enc()

    a, b = _run_threads(pinned, plain)
    assert torch.equal(a, ref) and torch.equal(b, ref)
    assert seen == {"a": "triple", "b_lib_is_product": True}
    assert D.jl_engine_for(10**7) == "single"  # this thread: auto


def test_prepared_factor_dropped_and_zeroed():
    """the node's prepared factor is zeroed and dropped by drop_prepared, by the
    clear-caches path and by an encrypt that raises; an encrypt of the prepared call still spends it."""
    from fedbiomed_amd.exceptions import FedbiomedSecaggCrypterError
    from fedbiomed_amd.secagg import SecaggCrypter

    P, tau, n, key = 3, 2, 2_000, W.jl_user_key(1)
    xl = W.party_params(1, n).astype(np.float64).tolist()
    jc = SecaggCrypter()
    ref = jc.encrypt(P, tau, xl, key, W.BIPRIME0, weight=5)
    for drop in ("method", "clear_caches", "encrypt_error"):
        assert jc.prepare_encrypt(tau, P, key, W.BIPRIME0, n)
        f = SecaggCrypter._enc_prep["factor"]
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(f)) > 0
        if drop == "method":
            SecaggCrypter.drop_prepared()
        elif drop == "clear_caches":
            D.jl_clear_caches()
        else:
            with pytest.raises(FedbiomedSecaggCrypterError):
                jc.encrypt(P, tau, xl, key, W.BIPRIME0, weight=2**17)  # the reference's weight error
        torch.cuda.synchronize()
        assert SecaggCrypter._enc_prep is None, drop
        assert int(torch.count_nonzero(f)) == 0, drop
    assert jc.prepare_encrypt(tau, P, key, W.BIPRIME0, n)
    assert jc.encrypt(P, tau, xl, key, W.BIPRIME0, weight=5) == ref and SecaggCrypter._enc_prep is None
    # the researcher's preparation: this instance's, dropped and zeroed alike
    assert jc.prepare_aggregate(tau, P, -key, W.BIPRIME0, n)
    fs = list(jc._prepared["factors"])
    jc.drop_prepared_aggregate()
    torch.cuda.synchronize()
    assert jc._prepared is None and all(int(torch.count_nonzero(f)) == 0 for f in fs)


def test_host_call_workspace_scrubbed():
    """after a synchronous host-buffer LOM call the device workspace holds no byte of the
    node's parameters or masked vector, and the clear-caches path releases every thread's workspace."""
    from fedbiomed_amd.secagg import SecaggLomCrypter

    P, tau, n = 3, 1, 1_000
    ids, ws = W.node_ids(P), [W.party_weight(p) for p in range(P)]
    lc = SecaggLomCrypter(W.LOM_NONCE)
    ys = [lc.encrypt(tau, u, W.party_params(p, n).astype(np.float64).tolist(), W.pairwise_secrets_for(u, ids), ids,
                     weight=ws[p]) for p, u in enumerate(ids)]
    torch.cuda.synchronize()
    wsp = D._host_ws[threading.get_ident()]
    assert int(torch.count_nonzero(wsp)) == 0
    lc.aggregate(ys, sum(ws))
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(wsp)) == 0
    D.jl_clear_caches()
    assert D._host_ws == {}


def test_four_threads_mixed_calls_soak():
    """Four threads at once, each repeating its own mix of list-API calls (a JL node encrypt, the JL researcher
    aggregate, a LOM encrypt and aggregate) at its own sizes and keys: every result equal to the same call made
    serially.  FBM_SOAK_ROUNDS repeats (default 2; round 6 ran 40 once: profiles/r6k_pytest_soak.txt)."""
    import os

    from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter

    rounds = int(os.environ.get("FBM_SOAK_ROUNDS", "2"))
    P, tau = 3, 5
    ids, ws = W.node_ids(P), [W.party_weight(p) for p in range(P)]

    def make(t):
        n = 700 + 911 * t  # different sizes per thread: different launches, strides and tails
        keys = [W.jl_user_key(10 * t + p) for p in range(P)]
        xs = [W.party_params(p + t, n).astype(np.float64).tolist() for p in range(P)]
        jc, lc = SecaggCrypter(), SecaggLomCrypter(W.LOM_NONCE)

        def call():
            cts = [jc.encrypt(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)]
            agg = jc.aggregate(tau, P, cts, -sum(keys), W.BIPRIME0, sum(ws), num_expected_params=n)
            ys = [lc.encrypt(tau, u, xs[p], W.pairwise_secrets_for(u, ids), ids, weight=ws[p])
                  for p, u in enumerate(ids)]
            lagg = lc.aggregate(ys, sum(ws))
            return cts, np.asarray(agg).view(np.uint64).tolist(), ys, np.asarray(lagg).view(np.uint64).tolist()

        return call

    calls = [make(t) for t in range(4)]
    refs = [c() for c in calls]
    for r in range(rounds):
        got = _run_threads(*calls)
        for t in range(4):
            assert got[t] == refs[t], (r, t)
