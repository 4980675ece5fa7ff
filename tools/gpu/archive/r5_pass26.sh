# round 5, pass 26: threaded in-place float writes -- the list aggregate at 10M x 8, plain and prepared, and the bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5at}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 16 --prepare-each > $O/list_agg_prepared.jsonl 2>&1 || { echo "PROBE FAILED"; tail -20 $O/list_agg_prepared.jsonl; exit 1; }
grep conv_threads $O/list_agg_prepared.jsonl
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); e=d['end_to_end']; r=e['researcher_aggregate_list_api']; print(d['value'], json.dumps(r['at_metric_size']), json.dumps(r['factor_prepared']), json.dumps(e['list_api']['prepared']), json.dumps(e['lom']['list_api']['output_prepared']))"
