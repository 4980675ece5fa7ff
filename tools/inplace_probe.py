#!/usr/bin/env python3
"""what the unprepared list calls gain from writing into output objects made ahead
(csrc/fbm_pyconv.c: int_pool + words_into_pool in the JL encrypt, the aggregate's last-stripe floats
made while the GPU exponentiates and then overwritten).  Times, interleaved, with
_device.INPLACE_UNPREPARED[call] on and off:
  * one node's SecaggCrypter.encrypt(List[float]) -> List[int] at --elements (the node's call),
  * the researcher's SecaggCrypter.aggregate(List[List[int]]) of P parties' lists at --elements,
each the median of --reps calls (the previous result freed outside the clock), outputs compared equal.
One JSON line per (call, setting), then a summary line.

    python tools/inplace_probe.py [--elements 10000000] [--reps 5]
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
    args = ap.parse_args()
    import numpy as np
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    P, tau, n = args.parties, 3, args.elements
    keys = [W.jl_user_key(p) for p in range(P)]
    ws = [W.party_weight(p) for p in range(P)]
    jc = SecaggCrypter()
    dev = D.device()
    xl0 = W.party_params(0, n).astype(np.float64).tolist()
    jc.encrypt(P, tau, xl0[:4096], keys[0], W.BIPRIME0, weight=ws[0])  # warm-up
    # the parties' ciphertext lists (made once, through the tensor API: the same values the list API gives)
    cl = []
    for p in range(P):
        ct = jc.encrypt_tensor(P, tau, torch.from_numpy(W.party_params(p, n)).to(dev), keys[p], W.BIPRIME0,
                               weight=ws[p])
        cl.append(D.limbs_to_ints(D.to_host(ct).numpy().view(np.uint32)))
    torch.cuda.synchronize()

    def enc():
        return jc.encrypt(P, tau, xl0, keys[0], W.BIPRIME0, weight=ws[0])

    def agg():
        return jc.aggregate(tau, P, cl, -sum(keys), W.BIPRIME0, sum(ws), num_expected_params=n)

    results, times = {}, {}
    for name, fn in (("node_encrypt", enc), ("researcher_aggregate", agg)):
        key = "encrypt" if name == "node_encrypt" else "aggregate"
        saved = dict(D.INPLACE_UNPREPARED)
        for setting in (True, False):
            D.INPLACE_UNPREPARED[key] = setting
            fn()  # a warm call of this setting
        for rep in range(args.reps):
            for setting in ((True, False) if rep % 2 == 0 else (False, True)):
                D.INPLACE_UNPREPARED[key] = setting
                res = None
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = fn()
                t = time.perf_counter() - t0
                times.setdefault((name, setting), []).append(t)
                if (name, setting) not in results:
                    results[(name, setting)] = res if name == "node_encrypt" else np.asarray(res).view(np.uint64)
                del res
        same = (results[(name, True)] == results[(name, False)]) if name == "node_encrypt" else bool(
            np.array_equal(results[(name, True)], results[(name, False)]))
        for setting in (True, False):
            ts = sorted(times[(name, setting)])
            print(json.dumps({"call": name, "inplace_unprepared": setting, "elements": n, "parties": P,
                              "median_ms": 1000 * ts[len(ts) // 2], "min_ms": 1000 * ts[0], "max_ms": 1000 * ts[-1],
                              "reps": len(ts), "equal_outputs": same}), flush=True)
        results.clear()
        D.INPLACE_UNPREPARED.update(saved)
    summ = {}
    for name in ("node_encrypt", "researcher_aggregate"):
        on = sorted(times[(name, True)])[args.reps // 2]
        off = sorted(times[(name, False)])[args.reps // 2]
        summ[name] = {"on_ms": 1000 * on, "off_ms": 1000 * off, "gain_pct": 100.0 * (off - on) / off}
    print(json.dumps({"summary": summ, "python": sys.version.split()[0], "inplace_allowed": D.inplace_allowed(),
                      "build_flags": list(D._pyconv().build_flags())}), flush=True)


if __name__ == "__main__":
    main()
