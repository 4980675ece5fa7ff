#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box: bench.py --gpus 2 spawns two ranks (gloo barrier /
# max-over-ranks; both ranks on cuda:0), strong split of 2M elements.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-dist}
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --elements 2000000 --steps 2 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e > $O/dist2.json 2> $O/dist2.err
rc=$?; echo rc=$rc; tail -c 600 $O/dist2.json; exit $rc
