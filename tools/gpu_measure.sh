#!/bin/bash
# One measurement pass on the GPU box (run through gpurun from the repo root):
# parity tests, the default bench line, a rocprofv3 kernel trace (+stats) and two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of the bench step, and the
# step of one rank of an 8-GPU strong split (the first 1/8 stripe of the 10M vector) on this GPU.
# Every GPU step has its own time limit; the chain stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r1}
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > $O/prof_bench.json 2> $O/prof.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $O/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $O/pmc_write.err &&
cd $R && timeout -k 10 300 python -u bench.py --elements 1250010 --steps 5 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e > $O/bench_stripe8.json 2> $O/bench_stripe8.err &&
if [ -x ./tools/microbench/madpeak ]; then timeout -k 10 120 ./tools/microbench/madpeak 400000 > $O/madpeak.txt 2>&1; fi
rc=$?
echo "rc=$rc"
tail -3 $O/pytest_gpu.txt
cat $O/bench.json $O/bench_stripe8.json
find $O -name "*.csv" | head -20
exit $rc
