# round 5, pass 10: prepare_aggregate (the crypter API GPU tests) and the bench line with the
# factor-ahead legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5q}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_crypter_api.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_crypter.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_crypter.txt; exit 1; }
tail -2 $O/pytest_crypter.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
