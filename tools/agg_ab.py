#!/usr/bin/env python3
"""LOM aggregate alone (fbm_lom_aggregate) at several (parties, elements) shapes, HIP events on the
launch stream (the library's own per-kernel events), median of 7: for A/B of library builds (FBM_LIB_PATH).  One JSON line per shape.

    FBM_AB_VARIANT=1 FBM_LIB_PATH=build/ab/x.so python tools/agg_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from fedbiomed_amd import _device as D, _native

    dev = D.device()
    for P, n in ((8, 10_000_000), (16, 10_000_000), (8, 100_000_000), (16, 100_000_000)):
        Y = torch.randint(0, 2**40, (P, n), dtype=torch.int64, device=dev)
        for sums in (False, True):
            ts = []
            for r in range(8):
                _native.prof_enable(r > 0)  # the library's per-kernel HIP events (the kernel alone)
                D.lom_aggregate(Y, 1000 * P, want_out=True, want_sums=sums)
                _native.prof_enable(False)
                rep = _native.prof_report()
                if r:
                    ts.append(rep["lom_aggregate"][1])
            ms = sorted(ts)[len(ts) // 2]
            b = 8 * (P + 1 + (1 if sums else 0)) * n
            print(json.dumps({"lib": os.path.basename(os.environ.get("FBM_LIB_PATH", "default")), "P": P, "n": n,
                              "sums": sums, "ms": round(ms, 4), "TBps": round(b / ms / 1e9, 3)}), flush=True)
        del Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
