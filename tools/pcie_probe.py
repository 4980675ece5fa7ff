#!/usr/bin/env python3
"""Host<->device copy rates from pinned memory (the list API's PCIe crossings): one copy of --mb MB on one
stream, and the same bytes split over 2 / 4 streams, each direction; median GB/s of --reps.

    python tools/pcie_probe.py [--mb 683] [--reps 5]
"""
import argparse
import json
import statistics
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=683)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    n = args.mb * 2**20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    res = {}
    for direction in ("h2d", "d2h"):
        for k in (1, 2, 4):
            streams = [torch.cuda.Stream() for _ in range(k)]
            ts = []
            for _ in range(args.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i, s in enumerate(streams):
                    a, b = n * i // k, n * (i + 1) // k
                    with torch.cuda.stream(s):
                        if direction == "h2d":
                            d[a:b].copy_(h[a:b], non_blocking=True)
                        else:
                            h[a:b].copy_(d[a:b], non_blocking=True)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            res[f"{direction}_{k}_streams_GBps"] = round(n / statistics.median(ts[1:]) / 1e9, 2)
    print(json.dumps({"bytes": n, **res}))


if __name__ == "__main__":
    main()
