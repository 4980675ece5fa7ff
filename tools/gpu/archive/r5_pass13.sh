# round 5, pass 13: the list aggregate with the GIL-held per-stripe conversion (no pins): crypter GPU tests,
# traces (prepared: fine stripes 65 536 and none; unprepared) and the probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5u}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_crypter_api.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_crypter.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_crypter.txt; exit 1; }
tail -2 $O/pytest_crypter.txt
for f in 131072; do
  FBM_FINE_STRIPE_CT=$f timeout -k 10 300 python -u tools/list_agg_trace.py --prepared --top 15 > $O/trace_prepared_$f.txt 2>&1 || { echo "TRACE $f FAILED"; tail -20 $O/trace_prepared_$f.txt; exit 1; }
  tail -1 $O/trace_prepared_$f.txt | cut -c1-300
done
timeout -k 10 300 python -u tools/list_agg_trace.py --top 15 > $O/trace_plain.txt 2>&1 || { echo "TRACE PLAIN FAILED"; exit 1; }
tail -1 $O/trace_plain.txt | cut -c1-300
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8 > $O/list_agg_probe.jsonl 2>&1 || { echo "PROBE FAILED"; exit 1; }
tail -1 $O/list_agg_probe.jsonl
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
