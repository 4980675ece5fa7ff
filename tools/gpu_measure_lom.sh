#!/bin/bash
# LOM measurement pass on the GPU box: rocprofv3 kernel trace (+stats) of the LOM bench
# (--scheme lom, 10M elements x 8 parties) and the two HBM PMC passes for its kernels.
# Summarise with: python tools/prof_summary.py gpurun_out/<tag> profiles/archive/r1_lom
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r1_lom}
mkdir -p $O
ARGS="--scheme lom --steps 5 --warmup 1 --serial --no-cpu-baseline --no-e2e"
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py $ARGS > $O/prof_bench.json 2> $O/prof.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $O/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py $ARGS > /dev/null 2> $O/pmc_write.err &&
cd $R && timeout -k 10 300 python bench.py --scheme lom --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc"
cat $O/bench.json
exit $rc
