#!/usr/bin/env python3
"""Where the aggregate step's time goes on one rank's stripe of an N-GPU split (N = 1, 2, 4, 8):
wall time of SecaggCrypter.aggregate_tensor (factor + combine, as bench.py's T_agg) and, in a
separate serialised pass, each kernel's HIP-event duration (fbm_prof_enable).

    python tools/agg_breakdown.py [--elements 10000000] [--parties 8] [--reps 5] [--engine auto]
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
    ap.add_argument("--elements", type=int, default=10_000_000)
    ap.add_argument("--parties", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--splits", default="1,2,4,8")
    ap.add_argument("--engine", default="auto")
    args = ap.parse_args()
    import torch

    from fedbiomed_amd import _device as D, _native, distributed, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau, n = args.parties, 1, args.elements
    keys = [W.jl_user_key(p) for p in range(P)]
    sk0 = -sum(keys)
    ws = [W.party_weight(p) for p in range(P)]
    jc = SecaggCrypter()
    es, cr = D.jl_slot(None, P)
    n_ct = (n + cr - 1) // cr
    xs = [torch.from_numpy(W.party_params(p, n)).to(dev) for p in range(P)]
    with D.jl_engine("single"):
        cts = torch.stack([jc.encrypt_tensor(P, tau, xs[p], keys[p], W.BIPRIME0, weight=ws[p]) for p in range(P)])
    del xs
    torch.cuda.synchronize()
    res = []
    with D.jl_engine(args.engine):
        for g in [int(v) for v in args.splits.split(",")]:
            hi = distributed.shard_range(n, g, 0, cr)[1]
            k = (hi + cr - 1) // cr
            part = cts if k == n_ct else cts[:, :k].contiguous()

            def agg():
                return jc.aggregate_tensor(tau, part, sk0, W.BIPRIME0, sum(ws), num_expected_params=hi)

            agg()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                agg()
                torch.cuda.synchronize()
                ts.append(1000 * (time.perf_counter() - t0))
            _native.prof_enable(True)
            agg()
            torch.cuda.synchronize()
            _native.prof_enable(False)
            kp = _native.prof_report()
            row = {"split": g, "elements": hi, "ciphertexts": k, "engine": D.jl_engine_for(k),
                   "wall_ms_median": sorted(ts)[len(ts) // 2], "wall_ms": [round(t, 3) for t in ts],
                   "kernels_ms": {name: round(t, 3) for name, (c, t) in sorted(kp.items())},
                   "kernels_sum_ms": round(sum(t for c, t in kp.values()), 3)}
            res.append(row)
            print(json.dumps(row), flush=True)
    whole = res[0]["wall_ms_median"] if res and res[0]["split"] == 1 else None
    if whole:
        print(json.dumps({"ratios": {r["split"]: round(whole / r["wall_ms_median"], 3) for r in res}}))


if __name__ == "__main__":
    main()
