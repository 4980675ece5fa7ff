#!/usr/bin/env python3
"""Drives the JL exponentiation alone for profiling: the decryption factor H(t_k)^sk0 of
`--ct` ciphertexts under each engine (rocprofv3 --kernel-trace / --pmc attribute the
dispatches to jl_exp_kernel / jl_expq_kernel).  Prints per-engine wall times.

    python tools/exp_probe.py [--ct 41667[,16384,...]] [--engines single,quad] [--reps 2] [--even]
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
    ap.add_argument("--ct", default="41667", help="comma-separated ciphertext counts")
    ap.add_argument("--engines", default="single,quad")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--even", action="store_true",
                    help="the even modulus BIPRIME0 + 1 (same width), which only the generic engine takes: timed as "
                         "powmods of caller-given odd bases (fbm_jl_powmod) -- an even N's FDH needs odd digests and "
                         "fails a ciphertext in 128 (the reference's OverflowError), so no large factor exists there")
    args = ap.parse_args()
    import torch

    from fedbiomed_amd import _device as D, workload as W

    dev = D.device()
    sk0 = W.jl_server_key(8)
    n = W.BIPRIME0 + 1 if args.even else W.BIPRIME0
    for ct in [int(c) for c in args.ct.split(",")]:
        out = {"ct": ct, "modulus": "even" if args.even else "odd"}
        if args.even:  # odd 256-bit bases, as one FDH digest would be
            g = torch.Generator().manual_seed(ct)
            h = torch.zeros((ct, 64), dtype=torch.int32)
            h[:, :8] = torch.randint(-2**31, 2**31 - 1, (ct, 8), generator=g, dtype=torch.int32)
            h[:, 0] |= 1
            h = h.to(dev)
            run = lambda: D.jl_powmod(h, n, abs(sk0))  # noqa: E731  (no inverse: a base may share a factor with N)
        else:
            run = lambda: D.jl_decrypt_factor(ct, n, sk0, 1, dev=dev)  # noqa: E731
        for eng in args.engines.split(","):
            with D.jl_engine(eng):
                run()
                torch.cuda.synchronize()
                ts = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    run()
                    torch.cuda.synchronize()
                    ts.append(round(1000 * (time.perf_counter() - t0), 3))
            out[eng + "_ms"] = ts
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
