#!/usr/bin/env python3
"""Engine co-scheduling probe: the decryption factor of n ciphertexts as ONE engine's launch
against a split -- the first `--single` ciphertexts on the one-lane engine and the rest on the
triple engine, the two launches on two HIP streams so their waves share the SIMDs (a one-lane wave
~236 VGPRs + a triple wave ~170 fit one SIMD's 512).  Prints wall times (median of reps).

    python tools/mixed_probe.py [--ct 83334] [--single 65536,49152,...] [--reps 5]
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
    ap.add_argument("--ct", default="83334,41667")
    ap.add_argument("--single", default="0,32768,49152,57344,65536,73728")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from fedbiomed_amd import _device as D, workload as W

    dev = D.device()
    sk0 = W.jl_server_key(8)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)
    for ct in [int(v) for v in args.ct.split(",")]:
        for ns in [int(v) for v in args.single.split(",")]:
            if ns > ct:
                continue

            def run():
                outs = []
                s1.wait_stream(main_s)
                s2.wait_stream(main_s)
                if ns:
                    with torch.cuda.stream(s1), D.jl_engine("single"):
                        outs.append(D.jl_decrypt_factor(ns, W.BIPRIME0, sk0, 1, dev=dev))
                if ct - ns:
                    with torch.cuda.stream(s2), D.jl_engine("triple"):
                        outs.append(D.jl_decrypt_factor(ct - ns, W.BIPRIME0, sk0, 1, ct_offset=ns, dev=dev))
                main_s.wait_stream(s1)
                main_s.wait_stream(s2)
                return outs

            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                run()
                torch.cuda.synchronize()
                ts.append(1000 * (time.perf_counter() - t0))
            print(json.dumps({"ct": ct, "single": ns, "triple": ct - ns, "ms": round(sorted(ts)[len(ts) // 2], 3),
                              "all": [round(t, 2) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
