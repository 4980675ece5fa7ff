# round 5 check pass: the -m gpu suite, smoke and the default bench line (one GPU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5a}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.txt; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
