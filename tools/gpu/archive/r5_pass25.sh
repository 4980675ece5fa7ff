# round 5, pass 25: the list aggregate's one-pass type check -- prepared probe and trace at 10M x 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5as}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 16 --prepare-each > $O/list_agg_prepared.jsonl 2>&1 || { echo "PROBE FAILED"; tail -20 $O/list_agg_prepared.jsonl; exit 1; }
grep conv_threads $O/list_agg_prepared.jsonl
timeout -k 10 300 python -u tools/list_agg_trace.py --prepared --top 12 > $O/trace_prepared.txt 2>&1 || { echo "TRACE FAILED"; tail -20 $O/trace_prepared.txt; exit 1; }
head -40 $O/trace_prepared.txt
