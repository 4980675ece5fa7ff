#!/usr/bin/env python3
"""Config 5 on one GPU (BASELINE.json configs[4]: LOM masking + additive secret sharing,
100M-element vector, 16 parties): the LOM step (every party's protect + the aggregate) and
the additive-sharing pair (split of the 100M summed vector into 16 int128 shares, exact
reconstruct), each timed with HIP events on the launch stream (median of --reps), with the
HBM rates of the two HBM-bound kernels against the 8 TB/s peak:
  lom_aggregate:   8 (P + 2) bytes per element (P u64 rows in, one f64 out, the u64 sum the
                   additive sharing splits)
  ass_reconstruct: 16 P + 16 bytes per element (P int128 shares in, one int128 sum out)
  ass_split:       8 + 16 P bytes per element (u64 in, P int128 shares out; ChaCha20 for the
                   P - 1 random shares).
An 8-GPU config-5 run splits the element range (8-aligned stripes, elem_offset): each rank
does 1/8 of this work with no collective.  Prints one JSON line.

    python tools/bench_cfg5.py [--elements 100000000] [--parties 16] [--reps 5]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=100_000_000)
    ap.add_argument("--parties", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import AdditiveSecret, AdditiveShares, SecaggLomCrypter

    dev = D.device()
    n, P, tau = args.elements, args.parties, 1
    ids, ws = W.node_ids(P), [W.party_weight(p) for p in range(P)]
    secrets_ = [W.pairwise_secrets_for(u, ids) for u in ids]
    cr = SecaggLomCrypter(W.LOM_NONCE)
    gen = torch.Generator(device=dev)
    xs = []
    for p in range(P):
        gen.manual_seed(500 + p)
        xs.append(torch.randn(n, generator=gen, device=dev, dtype=torch.float32) * 0.05)
    Y = torch.empty((P, n), dtype=torch.int64, device=dev)

    def timed(fn):
        fn()  # warm-up
        ts = []
        for _ in range(args.reps):
            s = torch.cuda.current_stream(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[len(ts) // 2]

    def protect_all():
        with D.deferred_checks():
            for p, u in enumerate(ids):
                cr.encrypt_tensor(tau, u, xs[p], secrets_[p], ids, weight=ws[p], out=Y[p])

    state = {}

    def aggregate():
        state["out"], state["sums"] = cr.aggregate_tensor(Y, sum(ws), want_sums=True)

    t_prot = timed(protect_all)
    t_agg = timed(aggregate)
    sums = state["sums"]
    del state["out"]

    def split():
        state["shares"] = AdditiveSecret.split_tensor(sums, P, unsigned=True)

    t_split = timed(split)
    shares = state["shares"]

    def reconstruct():
        state["rec"] = AdditiveShares.reconstruct_tensor(shares)

    t_rec = timed(reconstruct)
    ok = bool(torch.equal(state["rec"][:, 0], sums)) and bool((state["rec"][:, 1] == 0).all())

    def gbs(nbytes, ms):
        return nbytes / (ms / 1000) / 1e9

    agg_b, rec_b, split_b = 8 * (P + 2) * n, (16 * P + 16) * n, (8 + 16 * P) * n
    line = {
        "workload": f"config 5: LOM + additive secret sharing, {n:,} elements, {P} parties, 1 GPU",
        "lom_step": {"value": n / ((t_prot + t_agg) / 1000), "unit": "params/s", "ms": t_prot + t_agg,
                     "protect_all_ms": t_prot, "aggregate_ms": t_agg,
                     "aggregate_hbm_GBps": gbs(agg_b, t_agg), "aggregate_hbm_frac": gbs(agg_b, t_agg) / HBM_PEAK_GBS},
        "ass": {"split_ms": t_split, "split_GBps": gbs(split_b, t_split),
                "split_hbm_frac": gbs(split_b, t_split) / HBM_PEAK_GBS,
                "reconstruct_ms": t_rec, "reconstruct_GBps": gbs(rec_b, t_rec),
                "reconstruct_hbm_frac": gbs(rec_b, t_rec) / HBM_PEAK_GBS,
                "reconstruct_exact": ok},
        "note": "HIP events on the launch stream, median of reps; bytes: algorithmic (docstring)",
    }
    print(json.dumps(line))


if __name__ == "__main__":
    main()
