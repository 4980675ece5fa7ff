#!/usr/bin/env python3
"""Where the host time of the researcher's SecaggCrypter.aggregate(List[List[int]]) goes at the metric
size (10M elements, 8 parties): two warm calls, then one call under cProfile (top functions by own time,
the waits on the GPU included as `synchronize`), then per-stripe wall-clock marks of one more call taken
by wrapping the crypter's stripe helpers.  One JSON line.

    python tools/list_agg_trace.py [--elements 10000000] [--top 25]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=10_000_000)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--prepared", action="store_true", help="prepare_aggregate before every call (synchronised)")
    args = ap.parse_args()
    import numpy as np
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter
    from fedbiomed_amd.secagg import _secagg_crypter as SC

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

    def call():  # the previous result is freed before the clock starts (10M floats: ~50 ms to free)
        if args.prepared:
            assert jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = jc.aggregate(tau, P, lists, sk0, W.BIPRIME0, tw, num_expected_params=n)
        dt = 1000 * (time.perf_counter() - t0)
        del out
        return dt

    warm = [call(), call()]
    prof = cProfile.Profile()
    prof.enable()
    prof_ms = call()
    prof.disable()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(args.top)
    print(s.getvalue(), flush=True)

    marks = []
    t_start = [0.0]

    def mark(name, fn):
        def wrapped(*a, **k):
            t0 = time.perf_counter()
            r = fn(*a, **k)
            marks.append((name, round(1000 * (t0 - t_start[0]), 2), round(1000 * (time.perf_counter() - t0), 2)))
            return r
        return wrapped

    orig = (D.f64_into_list, D.convert_stripe, jc.decrypt_factor_tensor, jc.aggregate_tensor, SC._check_int_lists)
    D.f64_into_list = mark("floats", D.f64_into_list)
    D.convert_stripe = mark("convert(+floats)", D.convert_stripe)
    jc.decrypt_factor_tensor = mark("factor_issue", jc.decrypt_factor_tensor)
    jc.aggregate_tensor = mark("combine_issue", jc.aggregate_tensor)
    SC._check_int_lists = mark("check_int_lists", SC._check_int_lists)
    if args.prepared:
        assert jc.prepare_aggregate(tau, P, sk0, W.BIPRIME0, n)
    torch.cuda.synchronize()
    t_start[0] = time.perf_counter()
    out = jc.aggregate(tau, P, lists, sk0, W.BIPRIME0, tw, num_expected_params=n)
    total = 1000 * (time.perf_counter() - t_start[0])
    del out
    D.f64_into_list, D.convert_stripe, jc.decrypt_factor_tensor, jc.aggregate_tensor, SC._check_int_lists = orig
    print(json.dumps({"elements": n, "parties": P, "prepared": args.prepared,
                      "stripes": D.list_encrypt_stripes(len(lists[0]), dev),
                      "warm_ms": warm, "profiled_ms": prof_ms, "marked_ms": total,
                      "marks_name_start_ms_dur_ms": marks}), flush=True)


if __name__ == "__main__":
    main()
