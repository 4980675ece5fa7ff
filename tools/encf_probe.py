#!/usr/bin/env python3
"""One party's JL encrypt of a device-resident vector with its factor computed ahead (fbm_jl_encrypt_factor:
pack + one (N pt + 1) F product per ciphertext) against the exponentiation's encrypt, at 1M and 10M elements
(P = 8); wall ms by HIP events on the launch stream, median of reps; the two outputs compared.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel split.

    python tools/encf_probe.py [--elements 1000000,10000000] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", default="1000000,10000000")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from fedbiomed_amd import _device as D, workload as W
    from fedbiomed_amd.secagg import SecaggCrypter

    dev = D.device()
    jc = SecaggCrypter()
    P, tau, key = 8, 3, W.jl_user_key(0)
    for n in [int(v) for v in args.elements.split(",")]:
        x = torch.from_numpy(W.party_params(0, n)).to(dev)
        _, cr = D.jl_slot(None, P)
        n_ct = -(-n // cr)
        F = jc.decrypt_factor_tensor(tau, n_ct, key, W.BIPRIME0)
        ref = jc.encrypt_tensor(P, tau, x, key, W.BIPRIME0, weight=W.party_weight(0))
        out = torch.empty_like(ref)
        s = torch.cuda.current_stream(dev)
        times = {}
        for name, kw in (("factor_ahead", {"factor": F}), ("exponentiation", {})):
            ts = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                jc.encrypt_tensor(P, tau, x, key, W.BIPRIME0, weight=W.party_weight(0), out=out, **kw)
                b.record(s)
                b.synchronize()
                ts.append(a.elapsed_time(b))
            times[name] = statistics.median(ts)
            if name == "factor_ahead":
                equal = bool(torch.equal(out, ref))
        print(json.dumps({"elements": n, "ciphertexts": n_ct, "encrypt_factor_ahead_ms": times["factor_ahead"],
                          "encrypt_exponentiation_ms": times["exponentiation"], "equal": equal,
                          "params_per_s_factor_ahead": n / times["factor_ahead"] * 1e3}), flush=True)


if __name__ == "__main__":
    main()
