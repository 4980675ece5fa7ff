#!/bin/bash
# Only the rocprofv3 passes of tools/gpu_measure.sh (kernel trace + stats, FETCH_SIZE, WRITE_SIZE),
# each its own process under its own limit, on the serialised bench step (no stages).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py $A > $O/prof_bench.json 2> $O/prof.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py $A > /dev/null 2> $O/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py $A > /dev/null 2> $O/pmc_write.err
rc=$?; echo rc=$rc; exit $rc
