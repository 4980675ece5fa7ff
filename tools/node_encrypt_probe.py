#!/usr/bin/env python3
"""Where one node's SecaggCrypter.encrypt(List[float]) spends its time at 10M elements (the list API's
overlapped stripes, _secagg_crypter._encrypt_overlapped): host timestamps of every stripe's issue, of its
ciphertexts' arrival in the pinned buffer (the copy's event) and of the end of its int
conversion, against the whole call.  One JSON line per call.

    python tools/node_encrypt_probe.py [--elements 10000000] [--reps 3]"""

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
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import _secagg_crypter as SC

    rng = np.random.default_rng(5)
    xl = (rng.standard_normal(args.elements) * 0.05).astype(np.float32).astype(np.float64).tolist()
    jc = SC.SecaggCrypter()
    key, P, tau = W.jl_user_key(1), 8, 3
    jc.encrypt(P, tau, xl[:4096], key, W.BIPRIME0, weight=1)  # warm-up
    marks = []
    orig_ev, orig_conv, orig_pool = torch.cuda.Event.synchronize, D.limbs_to_ints, D.limbs_into_pool

    def ev_sync(self):
        orig_ev(self)
        marks.append(("arrived", time.perf_counter()))

    def conv(a):
        r = orig_conv(a)
        marks.append(("converted", time.perf_counter()))
        return r

    def into_pool(*a, **k):
        r = orig_pool(*a, **k)
        marks.append(("converted", time.perf_counter()))
        return r

    out = None
    for rep in range(args.reps + 1):
        out = None  # the previous call's ints freed outside the clock (a node keeps its result)
        marks.clear()
        torch.cuda.Event.synchronize, D.limbs_to_ints, D.limbs_into_pool = ev_sync, conv, into_pool
        try:
            t0 = time.perf_counter()
            out = jc.encrypt(P, tau, xl, key, W.BIPRIME0, weight=1)
            t1 = time.perf_counter()
        finally:
            torch.cuda.Event.synchronize, D.limbs_to_ints, D.limbs_into_pool = orig_ev, orig_conv, orig_pool
        if rep == 0:
            continue  # (the first full-size call allocates the pinned staging)
        n_ct = len(out)
        stripes = D.list_encrypt_stripes(n_ct)
        print(json.dumps({"elements": args.elements, "ciphertexts": n_ct, "stripes": stripes, "ms": 1000 * (t1 - t0),
                          "marks_ms": [(k, round(1000 * (t - t0), 2)) for k, t in marks]}), flush=True)


if __name__ == "__main__":
    main()
