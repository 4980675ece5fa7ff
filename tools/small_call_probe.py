#!/usr/bin/env python3
"""Where a small list-API call's time goes (BASELINE config 1: LOM, 1 000 elements, 2 parties): the
encrypt and the aggregate in their host-side steps, median of --reps microseconds each, after a warm-up.

    python tools/small_call_probe.py [--elements 1000] [--reps 200]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggLomCrypter

    n, P = args.elements, 2
    ids = W.node_ids(P)
    lc = SecaggLomCrypter("small_call")
    xs = [np.random.default_rng(p).uniform(-1, 1, n).tolist() for p in range(P)]
    sec = W.pairwise_secrets_for(ids[0], ids)
    dev = D.device()
    steps = {k: [] for k in ("floats_to_host", "h2d", "protect_and_check", "d2h", "tolist", "encrypt_call",
                             "aggregate_call", "protect_host_call", "aggregate_host_call", "peer_masks")}
    ys = [lc.encrypt(1, u, xs[p], W.pairwise_secrets_for(u, ids), ids, weight=7) for p, u in enumerate(ids)]
    Yh = np.array(ys, dtype=np.uint64)
    for _ in range(args.reps):
        t0 = time.perf_counter()
        host = D.floats_to_host(xs[0])
        t1 = time.perf_counter()
        x = host.to(dev)
        t2 = time.perf_counter()
        y = lc.encrypt_tensor(1, ids[0], x, sec, ids, weight=7)
        t3 = time.perf_counter()
        packed = D.to_host(y).numpy().view(np.uint64)
        t4 = time.perf_counter()
        packed.tolist()
        t5 = time.perf_counter()
        lc.encrypt(1, ids[0], xs[0], sec, ids, weight=7)
        t6 = time.perf_counter()
        lc.aggregate(ys, 14)
        t7 = time.perf_counter()
        sm, sg = lc._peer_masks(ids[0], sec, ids)
        t8 = time.perf_counter()
        D.lom_protect_host(host.numpy(), sm, sg, lc.nonce, 1, P, weight=7)
        t9 = time.perf_counter()
        D.lom_aggregate_host(Yh, 14)
        t10 = time.perf_counter()
        for k, a, b in (("floats_to_host", t0, t1), ("h2d", t1, t2), ("protect_and_check", t2, t3), ("d2h", t3, t4),
                        ("tolist", t4, t5), ("encrypt_call", t5, t6), ("aggregate_call", t6, t7), ("peer_masks", t7, t8),
                        ("protect_host_call", t8, t9), ("aggregate_host_call", t9, t10)):
            steps[k].append(1e6 * (b - a))
    torch.cuda.synchronize()
    print(json.dumps({"elements": n, "median_us": {k: round(statistics.median(v), 1) for k, v in steps.items()}}))


if __name__ == "__main__":
    main()
