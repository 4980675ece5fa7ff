#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box: bench.py --gpus N spawns N ranks (gloo barrier /
# max-over-ranks; all ranks on cuda:0), strong split of 2M elements, every default leg the driver's
# N > 1 runs take (the JL step, stages, the LOM leg on its own 8-aligned stripes).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-dist}
mkdir -p $O
cd $R
for g in 2 4; do
  timeout -k 10 300 python -u bench.py --gpus $g --dist-backend gloo --elements 2000000 --steps 2 --warmup 1 \
    > $O/dist$g.json 2> $O/dist$g.err || { rc=$?; echo "gpus=$g rc=$rc"; tail -c 1500 $O/dist$g.err; exit $rc; }
  tail -c 300 $O/dist$g.json; echo
done
