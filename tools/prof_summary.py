#!/usr/bin/env python3
"""Summarise a rocprofv3 measurement pass (tools/gpu_measure.sh) into profiles/.

    python tools/prof_summary.py gpurun_out/r2 profiles/archive/r1

reads  <dir>/prof      (--kernel-trace --stats)   -> <prefix>_kernel_stats.csv
       <dir>/pmc_fetch (--pmc FETCH_SIZE)          -> <prefix>_hbm_traffic.json
       <dir>/pmc_write (--pmc WRITE_SIZE)
Both the CSV and the SQLite (rocpd) output formats of rocprofv3 are understood.

HBM traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes), following
/opt/skills/guides/MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of a
coalesced streaming read, WRITE_SIZE reads exactly; the two counters need separate passes.
"""

import collections
import csv
import glob
import json
import os
import sqlite3
import sys


def _short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").strip()


def _dispatches(d: str):
    """[(kernel, duration_ns)] from a --kernel-trace output directory."""
    out = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                out.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    if out:
        return out
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        out += [(n, int(du)) for n, du in c.execute("select name, duration from kernels")]
    return out


def _counters(d: str, counter: str):
    """{kernel: [value per dispatch]} from a --pmc output directory."""
    agg = collections.defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter:
                    agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    if files:
        return agg
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        for k, v in c.execute("select kernel_name, value from counters_collection where counter_name = ?",
                              (counter,)):
            agg[k].append(float(v))
    return agg


def main(src: str, prefix: str) -> None:
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    disp = _dispatches(os.path.join(src, "prof"))
    stats = collections.defaultdict(list)
    for n, du in disp:
        stats[_short(n)].append(du)
    total = sum(sum(v) for v in stats.values()) or 1
    rows = sorted(((k, len(v), sum(v) / 1e6, sum(v) / len(v) / 1e6, min(v) / 1e6, max(v) / 1e6,
                    100.0 * sum(v) / total) for k, v in stats.items()), key=lambda r: -r[2])
    with open(prefix + "_kernel_stats.csv", "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "calls", "total_ms", "avg_ms", "min_ms", "max_ms", "percent"])
        for r in rows:
            w.writerow([r[0], r[1]] + [f"{x:.4f}" for x in r[2:]])
    fetch = _counters(os.path.join(src, "pmc_fetch"), "FETCH_SIZE")
    write = _counters(os.path.join(src, "pmc_write"), "WRITE_SIZE")
    traffic = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        wv = write.get(k, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(wv) / len(wv) if wv else 0.0
        traffic[_short(k)] = {"launches": max(len(f), len(wv)), "FETCH_SIZE_KB": fk, "WRITE_SIZE_KB": wk,
                              "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0}
    meta = {"source": src, "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950, MI355X_MICROARCH.md)"}
    if os.path.exists(os.path.join(src, "prof_bench.json")):
        try:
            with open(os.path.join(src, "prof_bench.json")) as fh:
                meta["bench_config"] = json.loads(fh.read().strip().splitlines()[-1]).get("config")
        except (ValueError, IndexError):
            pass
    with open(prefix + "_hbm_traffic.json", "w") as fh:
        json.dump({"meta": meta, "kernels": traffic}, fh, indent=1)
    for r in rows[:12]:
        print(f"{r[0]:40s} calls {r[1]:4d} total {r[2]:10.2f} ms avg {r[3]:9.3f} ms {r[6]:5.1f}%")
    for k, v in traffic.items():
        print(f"{k:40s} HBM/launch {v['hbm_bytes_per_launch'] / 1e6:10.1f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
