# round 5, pass 29: BASELINE configs 1-3 through the list API, plain and prepared, beside the reference's CPU times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ax}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/bench_configs.py > $O/bench_configs.jsonl 2> $O/bench_configs.err || { echo "CONFIGS FAILED"; tail -20 $O/bench_configs.err; exit 1; }
cat $O/bench_configs.jsonl
