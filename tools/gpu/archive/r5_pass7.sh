# round 5, pass 7: where the researcher list aggregate's host time goes (cProfile + per-stripe marks),
# then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5k}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/list_agg_trace.py > $O/list_agg_trace.txt 2>&1 || { echo "LIST AGG TRACE FAILED"; tail -20 $O/list_agg_trace.txt; exit 1; }
tail -1 $O/list_agg_trace.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
