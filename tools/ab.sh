#!/bin/bash
# A/B timing of library variants on one box (variants built beforehand, in this container:
#   python -m fedbiomed_amd._build --out build/ab/<name>.so -D...).
# usage (on the GPU box): bash tools/ab.sh <outdir> "<bench args>" name1 name2 ...
# Runs every variant twice, interleaved (A B C A B C), each under its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
ARGS=$1; shift
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in "$@"; do
    FBM_AB_VARIANT=1 FBM_LIB_PATH=$R/build/ab/$v.so timeout -k 10 300 python bench.py $ARGS > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "FAIL $v"; tail -5 $O/$v.$rep.err; exit 1; }
    python - "$O/$v.$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["total_ms"] / v["launches"], 4) for n, v in d.get("kernels_ms", {}).items()}
print(f"{sys.argv[2]:>14} value {d['value']:.4g}  ms/step {d['ms_per_step']:.3f}  per-launch ms {k}")
PY
  done
done
