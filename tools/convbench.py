#!/usr/bin/env python3
"""Host conversion rates of the list API (csrc/fbm_pyconv.c) at the bench's list-leg size:
8 parties x 33 334 JL ciphertexts (1M elements at P = 8), per thread count.

    python tools/convbench.py [threads ...]      (FBM_CONV_THREADS per run; CPU only)
"""
import json
import os
import random
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one():
    sys.path.insert(0, ROOT)
    import numpy as np

    from fedbiomed_amd import _device as D, workload as W

    m = D._pyconv()
    rng = random.Random(1)
    n = 33334 * 8
    cts = [rng.randrange(W.BIPRIME0 ** 2) for _ in range(n)]
    out = np.zeros((n, 64), np.uint32)
    best = [1e9, 1e9]
    for _ in range(5):
        t0 = time.perf_counter()
        assert m.ints_to_bytes(cts, 256, out) == -1
        t1 = time.perf_counter()
        back = m.bytes_to_ints(out, 256)
        t2 = time.perf_counter()
        best = [min(best[0], t1 - t0), min(best[1], t2 - t1)]
        del back
    print(json.dumps({"threads": os.environ.get("FBM_CONV_THREADS", "8"), "ciphertexts": n,
                      "ints_to_bytes_ms": round(1e3 * best[0], 2), "bytes_to_ints_ms": round(1e3 * best[1], 2)}))


if __name__ == "__main__":
    if os.environ.get("_FBM_CONVBENCH_CHILD"):
        one()
    else:
        for t in sys.argv[1:] or ["1", "8", "16"]:
            env = dict(os.environ, FBM_CONV_THREADS=t, _FBM_CONVBENCH_CHILD="1")
            subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, check=True)
