#!/usr/bin/env python3
"""BASELINE configs 1-3 through the reference's own API on one GPU, beside the reference's CPU times that
BASELINE.md holds for the same inputs (float32 uniform in [-1, 1), weight 7, tau = 1, clipping 3, target
2**13; JL keys of 2040 bits on biprime0): every party's `encrypt(List[float]) -> List[int]`, then the
researcher's `aggregate`, wall time from host lists to host lists -- plain, and with each call prepared
(`prepare_encrypt` / `prepare_aggregate`, extensions; their work outside the clock, as while the nodes
train).  Best of --reps after a warm-up; the outputs compared with the plain calls'.  One JSON line per
config.

    python tools/bench_configs.py [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# BASELINE.md, "Reference CPU numbers measured in the survey container": encrypt all parties / aggregate, s
REFERENCE_S = {1: (0.88e-3, 0.21e-3), 2: (18.46, 4.75), 3: (3.08, 0.34)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from fedbiomed_amd import workload as W
    from fedbiomed_amd.secagg import SecaggCrypter, SecaggLomCrypter

    rng = np.random.default_rng(1)
    weight, tau, clip, target = 7, 1, 3, 2**13
    for cfg, scheme, n, P in ((1, "lom", 1000, 2), (2, "jl", 100_000, 4), (3, "lom", 1_199_882, 4)):
        xs = [rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64).tolist() for _ in range(P)]
        ids = W.node_ids(P)
        if scheme == "jl":
            keys = [W.jl_user_key(p) for p in range(P)]
            sk0 = -sum(keys)
            jc = SecaggCrypter()

            def enc(p, prep):
                if prep:
                    jc.prepare_encrypt(tau, P, keys[p], W.BIPRIME0, n)
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                c = jc.encrypt(P, tau, xs[p], keys[p], W.BIPRIME0, clipping_range=clip, weight=weight,
                               target_range=target)
                return c, time.perf_counter() - t0

            def agg(cts, prep):
                if prep:
                    jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n, target_range=target)
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                out = jc.aggregate(tau, P, cts, sk0, W.BIPRIME0, P * weight, clipping_range=clip,
                                   num_expected_params=n, target_range=target)
                return out, time.perf_counter() - t0
        else:
            lc = SecaggLomCrypter("bench_configs")

            def enc(p, prep):
                u = ids[p]
                if prep:
                    lc.prepare_encrypt(tau, u, n)
                t0 = time.perf_counter()
                y = lc.encrypt(tau, u, xs[p], W.pairwise_secrets_for(u, ids), ids, clipping_range=clip,
                               weight=weight, target_range=target)
                return y, time.perf_counter() - t0

            def agg(ys, prep):
                if prep:
                    lc.prepare_aggregate(n)
                t0 = time.perf_counter()
                out = lc.aggregate(ys, P * weight, clipping_range=clip, target_range=target)
                return out, time.perf_counter() - t0

        res = {}
        ref_out = None
        for prep in (False, True):
            best_e, best_a, equal = 1e9, 1e9, True
            for rep in range(args.reps + 1):
                cts, te = [], 0.0
                for p in range(P):
                    c, t = enc(p, prep)
                    cts.append(c)
                    te += t
                out, ta = agg(cts, prep)
                if ref_out is None:
                    ref_out, ref_cts = out, cts
                equal &= out == ref_out and cts == ref_cts
                if rep:  # (the first call warms the staging buffers and the key caches)
                    best_e, best_a = min(best_e, te), min(best_a, ta)
                del cts, out
            res["prepared" if prep else "plain"] = {"encrypt_all_ms": 1e3 * best_e, "aggregate_ms": 1e3 * best_a,
                                                    "total_ms": 1e3 * (best_e + best_a), "equal": equal}
        re, ra = REFERENCE_S[cfg]
        line = {"config": cfg, "scheme": scheme, "elements": n, "parties": P, **res,
                "reference_cpu_ms": {"encrypt_all": 1e3 * re, "aggregate": 1e3 * ra, "total": 1e3 * (re + ra),
                                     "source": "BASELINE.md (1 EPYC core, the reference through its shims)"},
                "speedup_plain": (re + ra) / (res["plain"]["total_ms"] / 1e3),
                "speedup_prepared": (re + ra) / (res["prepared"]["total_ms"] / 1e3)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
