#!/usr/bin/env python3
"""Calibrate the bench's CPU baseline: time the REFERENCE crypter (imported from
/root/reference through tools/refshim) and the oracle restatement
(oracle/secagg_oracle.py) on the identical sample the bench's `cpu_baseline` leg uses
(bench.py: 20k elements x 8 parties, JL encrypt all + aggregate; LOM 500k x 8), single
thread, in this container.  The reference never travels to the GPU box, so the bench
reports the oracle it times there and, from this committed ratio, the reference-equivalent
rate (`cpu_baseline.reference_equivalent`).

    python tools/calibrate_cpu.py      -> profiles/cpu_calibration.json
"""

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "refshim"))
sys.path.insert(0, REPO)

import load_reference  # noqa: E402

from fedbiomed_amd import workload as W  # noqa: E402
from oracle import secagg_oracle as O  # noqa: E402


def jl_sample(ns, P, tau=1):
    xs = [[float(v) for v in W.party_params(p, ns)] for p in range(P)]
    keys = [W.jl_user_key(p) for p in range(P)]
    ws = [W.party_weight(p) for p in range(P)]
    return xs, keys, ws, -sum(keys)


def time_jl(R, ns, P, tau=1):
    xs, keys, ws, sk0 = jl_sample(ns, P, tau)
    t0 = time.perf_counter()
    cts = [O.jl_encrypt(xs[p], tau, keys[p], W.BIPRIME0, P, weight=ws[p]) for p in range(P)]
    O.jl_crypter_aggregate(cts, tau, sk0, W.BIPRIME0, sum(ws), ns)
    t_oracle = time.perf_counter() - t0
    C = R.crypter.SecaggCrypter
    t0 = time.perf_counter()
    rc = [C().encrypt(num_nodes=P, current_round=tau, params=xs[p], key=keys[p], biprime=W.BIPRIME0, weight=ws[p])
          for p in range(P)]
    C().aggregate(current_round=tau, num_nodes=P, params=rc, key=sk0, biprime=W.BIPRIME0, total_sample_size=sum(ws),
                  num_expected_params=ns)
    t_ref = time.perf_counter() - t0
    assert [int(c) for c in rc[0]] == cts[0], "reference and oracle ciphertexts differ"
    return t_ref, t_oracle


def time_lom(R, ns, P, tau=1):
    ids = W.node_ids(P)
    xs = [[float(v) for v in W.party_params(p, ns)] for p in range(P)]
    ws = [W.party_weight(p) for p in range(P)]
    sec = [W.pairwise_secrets_for(u, ids) for u in ids]
    non = O.lom_nonce(W.LOM_NONCE)
    t0 = time.perf_counter()
    ys = [O.lom_encrypt(xs[p], tau, u, sec[p], ids, non, weight=ws[p]) for p, u in enumerate(ids)]
    O.lom_crypter_aggregate(ys, sum(ws))
    t_oracle = time.perf_counter() - t0
    C = R.crypter.SecaggLomCrypter
    t0 = time.perf_counter()
    ry = [C(W.LOM_NONCE).encrypt(current_round=tau, node_id=u, params=xs[p], pairwise_secrets=sec[p], node_ids=ids,
                                 weight=ws[p]) for p, u in enumerate(ids)]
    C(W.LOM_NONCE).aggregate(params=ry, total_sample_size=sum(ws))
    t_ref = time.perf_counter() - t0
    assert [int(v) for v in ry[0]] == [int(v) for v in ys[0]], "reference and oracle LOM vectors differ"
    return t_ref, t_oracle


def main():
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    R = load_reference.load()
    P = 8
    out = {"generator": "tools/calibrate_cpu.py", "threads": 1, "parties": P,
           "host": "build container (8 vCPU AMD EPYC), one core"}
    for scheme, ns, fn in (("jl", 20_000, time_jl), ("lom", 500_000, time_lom)):
        t_ref, t_or = fn(R, ns, P)
        out[scheme] = {"elements": ns, "reference_s": t_ref, "oracle_s": t_or,
                       "reference_params_per_s": ns / t_ref, "oracle_params_per_s": ns / t_or,
                       "reference_over_oracle_time": t_ref / t_or}
        print(scheme, json.dumps(out[scheme]))
    path = os.path.join(REPO, "profiles", "cpu_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
