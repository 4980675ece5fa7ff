# round 5, pass 32: one synchronisation fewer per list call -- the GPU suite, then the small-call probe and configs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bb}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" $O/pytest_gpu.txt | head -30; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 200 python -u tools/small_call_probe.py > $O/small_call.jsonl 2> $O/small_call.err || { echo "PROBE FAILED"; tail -20 $O/small_call.err; exit 1; }
cat $O/small_call.jsonl
timeout -k 10 300 python -u tools/bench_configs.py > $O/bench_configs.jsonl 2> $O/bench_configs.err || { echo "CONFIGS FAILED"; tail -20 $O/bench_configs.err; exit 1; }
cut -c1-330 $O/bench_configs.jsonl
