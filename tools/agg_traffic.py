#!/usr/bin/env python3
"""Summarise tools/pmc_agg.sh: per aggregate-side kernel, the average launch time and the
HBM traffic per launch (2 * FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md) against the
algorithmic bytes of DESIGN.md section 4, at the full vector and at the 1/8 stripe.

    python tools/agg_traffic.py gpurun_out/pmcagg2 profiles/archive/r2_s4_agg_traffic.json
"""

import collections
import csv
import json
import sys

P = 8
SIZES = {"10000000": 333334, "1250010": 41667}
ALGO = {  # bytes per ciphertext
    "fbm::jl_prod_kernel": 256 * (P + 1) + 128,
    "fbm::jl_lift_kernel": 256 + 128 + 256,
    "fbm::jl_inv_modn_kernel": 128 + 128,
    "fbm::jl_fdh_kernel": 256,
    "fbm::jl_decode_kernel": 128 + 30 * 8,
}


def _short(name):
    return name.split("(")[0].replace("void ", "").strip()


def _counter(path):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        acc[(_short(r["Kernel_Name"]), r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (k, _), v in acc.items():
        per[k].append(v)
    return {k: sum(v) / len(v) for k, v in per.items()}


def main(src, dst):
    out = {"meta": {"source": src, "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950)",
                    "parties": P, "algorithmic_bytes_per_ct": ALGO}}
    for n, nct in SIZES.items():
        fetch, write = _counter(f"{src}/fetch_{n}/run_counter_collection.csv"), \
            _counter(f"{src}/write_{n}/run_counter_collection.csv")
        dur = {_short(r["Name"]): float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(f"{src}/kt_{n}/run_kernel_stats.csv"))}
        rows = {}
        for k, per_ct in ALGO.items():
            if k not in fetch:
                continue
            hbm = (2 * fetch[k] + write.get(k, 0.0)) * 1024
            rows[k] = {"avg_ms": dur.get(k), "hbm_bytes_per_launch": hbm, "algorithmic_bytes": per_ct * nct,
                       "ratio": hbm / (per_ct * nct)}
        out[f"elements_{n}"] = {"ciphertexts": nct, "kernels": rows}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for n in SIZES:
        for k, r in out[f"elements_{n}"]["kernels"].items():
            print(n, k, f"{r['avg_ms']:.3f} ms", f"{r['hbm_bytes_per_launch'] / 1e6:.1f} MB", f"x{r['ratio']:.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
