#!/usr/bin/env python3
"""Aggregate-step strong-scaling probe on ONE GPU.

Times the JL aggregate alone -- decryption factor H(t_k)^sk0 (FDH + exponentiation +
inverse) and the combine (ciphertext product, (v-1)/N, decode, average, dequantise) -- at a
whole config-4 vector (10M elements, 8 parties) and at the stripe one of 8 GPUs owns
(1.25M elements), and one party's encrypt at the same two sizes.  The ratio
T(10M) / T(1.25M) is the 8-GPU speed-up the step can reach when the element range is split
(SURVEY §8(e)); the north star asks >= 6x for the aggregate step.

    python tools/agg_scaling.py [--engine auto|single|quad] [--reps 3]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="10000000,1250000")
    ap.add_argument("--parties", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--engine", default=None, help="auto | single | quad (library default if omitted)")
    args = ap.parse_args()
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau = args.parties, 1
    keys = [W.jl_user_key(p) for p in range(P)]
    sk0 = -sum(keys)
    ws = [W.party_weight(p) for p in range(P)]
    jc = SecaggCrypter()
    es, cr = D.jl_slot(None, P)
    res = {"parties": P, "engine": args.engine or "library default"}
    ctx = D.jl_engine(args.engine) if args.engine and hasattr(D, "jl_engine") else None
    if ctx is not None:
        ctx.__enter__()
    for n in [int(s) for s in args.sizes.split(",")]:
        n_ct = (n + cr - 1) // cr
        xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
        cts = torch.stack([jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)])

        def agg():
            f = jc.decrypt_factor_tensor(tau, n_ct, sk0, W.BIPRIME0)
            return jc.aggregate_tensor(tau, cts, sk0, W.BIPRIME0, sum(ws), num_expected_params=n, decrypt_factor=f)

        def enc1():
            return jc.encrypt_tensor(P, tau, xs[0], keys[0], W.BIPRIME0, weight=ws[0])

        row = {"elements": n, "ciphertexts": n_ct}
        for name, fn in (("aggregate_ms", agg), ("encrypt_one_party_ms", enc1)):
            fn()
            torch.cuda.synchronize()
            t = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                t.append(1000 * (time.perf_counter() - t0))
            row[name] = min(t)
            row[name + "_all"] = [round(v, 2) for v in t]
        res[str(n)] = row
        print(json.dumps(row), flush=True)
        del xs, cts
    sz = [int(s) for s in args.sizes.split(",")]
    if len(sz) == 2:
        a, b = res[str(sz[0])], res[str(sz[1])]
        res["aggregate_ratio"] = a["aggregate_ms"] / b["aggregate_ms"]
        res["encrypt_ratio"] = a["encrypt_one_party_ms"] / b["encrypt_one_party_ms"]
    if ctx is not None:
        ctx.__exit__(None, None, None)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
