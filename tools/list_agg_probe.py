#!/usr/bin/env python3
"""The researcher's SecaggCrypter.aggregate(List[List[int]]) at the metric size (10M elements, 8 parties:
8 x 333 334 ciphertexts as Python ints) under several host-conversion thread counts (FBM_CONV_THREADS, read
per call by csrc/fbm_pyconv.c), best of 3 calls each, with the conversion and the output float list alone beside it.  One JSON line
per thread count.

    python tools/list_agg_probe.py [--threads 4,8,16] [--elements 10000000] [--first-call plain|prepared]
                                   [--prepare-each]
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
    ap.add_argument("--threads", default="4,8,16")
    ap.add_argument("--elements", type=int, default=10_000_000)
    ap.add_argument("--first-call", choices=("plain", "prepared"), default=None,
                    help="time only the process's first aggregate, with or without prepare_aggregate before it")
    ap.add_argument("--prepare-each", action="store_true",
                    help="prepare_aggregate before every timed call (outside the clock, then a sync: the nodes' "
                         "training time)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    P, tau, n = 8, 3, args.elements
    keys = [W.jl_user_key(p) for p in range(P)]
    sk0 = -sum(keys)
    jc = SecaggCrypter()
    lists = []
    for p in range(P):
        x = torch.from_numpy(W.party_params(p, n)).to(dev)
        ct = jc.encrypt_tensor(P, tau, x, keys[p], W.BIPRIME0, weight=W.party_weight(p))
        lists.append(D.limbs_to_ints(D.to_host(ct).numpy().view(np.uint32)))
        del ct, x
    tw = sum(W.party_weight(p) for p in range(P))
    n2 = W.BIPRIME0 * W.BIPRIME0
    if args.first_call:  # the first aggregate of a fresh crypter process (a researcher's first round)
        prepared = jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n) if args.first_call == "prepared" else False
        torch.cuda.synchronize()  # (the nodes' training time)
        t0 = time.perf_counter()
        jc.aggregate(tau, P, lists, sk0, W.BIPRIME0, tw, num_expected_params=n)
        t = time.perf_counter() - t0
        print(json.dumps({"first_call": args.first_call, "prepared": prepared, "elements": n, "parties": P,
                          "aggregate_ms": 1000 * t}), flush=True)
        return
    ref = None
    for t in [int(v) for v in args.threads.split(",")]:
        os.environ["FBM_CONV_THREADS"] = str(t)
        conv = []
        for _ in range(3):
            t0 = time.perf_counter()
            staged = D.host_empty((P, len(lists[0]), 64), torch.int32)
            limbs = staged.numpy().view(np.uint32)
            for u in range(P):
                D.ints_to_limbs(lists[u], n2, out=limbs[u])
            conv.append(time.perf_counter() - t0)
        calls = []
        for _ in range(3):
            out = None  # the previous call's list is freed outside the clock
            if args.prepare_each:
                assert jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = jc.aggregate(tau, P, lists, sk0, W.BIPRIME0, tw, num_expected_params=n)
            calls.append(time.perf_counter() - t0)
        ref = out if ref is None else ref
        floats = []
        res_h = np.asarray(out, dtype=np.float64)
        for _ in range(3):
            t0 = time.perf_counter()
            lst = res_h.tolist()
            floats.append(time.perf_counter() - t0)
            del lst
        print(json.dumps({"conv_threads": t, "prepared": args.prepare_each, "elements": n, "parties": P, "aggregate_ms": 1000 * min(calls),
                          "aggregate_ms_all": [1000 * c for c in calls],
                          "params_per_s": n / min(calls), "conversion_alone_ms": 1000 * min(conv),
                          "float_list_alone_ms": 1000 * min(floats),
                          "equal_across_thread_counts": out == ref}), flush=True)


if __name__ == "__main__":
    main()
