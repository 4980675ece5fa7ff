# round 5, pass 8: the -m gpu suite, then the researcher list aggregate with the background int
# conversion and the in-place float list (trace + probe)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5l}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -u tools/list_agg_trace.py > $O/list_agg_trace.txt 2>&1 || { echo "LIST AGG TRACE FAILED"; tail -20 $O/list_agg_trace.txt; exit 1; }
tail -1 $O/list_agg_trace.txt
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8 > $O/list_agg_probe.jsonl 2>&1 || { echo "LIST AGG PROBE FAILED"; tail -5 $O/list_agg_probe.jsonl; exit 1; }
tail -1 $O/list_agg_probe.jsonl
