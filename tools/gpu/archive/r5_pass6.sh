# round 5, pass 6: the -m gpu suite and the striped researcher list aggregate at the metric size
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5i}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8 > $O/list_agg_probe.jsonl 2>&1 || { echo "LIST AGG PROBE FAILED"; tail -5 $O/list_agg_probe.jsonl; exit 1; }
tail -1 $O/list_agg_probe.jsonl
FBM_ONE_LANE_ROUND=100000000 timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8 > $O/list_agg_probe_unsplit.jsonl 2>&1 || { echo "LIST AGG PROBE (unsplit) FAILED"; exit 1; }
tail -1 $O/list_agg_probe_unsplit.jsonl
