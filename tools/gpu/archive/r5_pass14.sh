# round 5, pass 14: host-thread count of the list aggregate's conversions (8 vs 16: the box's CPU share)
# and the bench line after the GIL-held ints_to_bytes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ab}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8,16,12 > $O/list_agg_probe.jsonl 2>&1 || { echo "PROBE FAILED"; tail -5 $O/list_agg_probe.jsonl; exit 1; }
grep conv_threads $O/list_agg_probe.jsonl
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
tail -c 200 $O/bench.json
