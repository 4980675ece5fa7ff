# round 5, pass 3: config 5's kernel trace + HBM-traffic passes with the wave-split kernels, then the
# one-GPU strong-scaling prediction (tools/predict_scaling.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5f}
mkdir -p $O/cfg5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg5/prof -o run -- python3 $R/tools/bench_cfg5.py --reps 1 > $O/cfg5/prof_bench.json 2> $O/cfg5/prof.err &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cfg5/pmc_fetch -o run -- python3 $R/tools/bench_cfg5.py --reps 1 > /dev/null 2> $O/cfg5/fetch.err &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cfg5/pmc_write -o run -- python3 $R/tools/bench_cfg5.py --reps 1 > /dev/null 2> $O/cfg5/write.err || { echo "CFG5 PROF FAILED"; exit 1; }
cd $R
bash tools/predict_scaling.sh ${1:-r5f}
