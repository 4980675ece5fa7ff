# round 4: the -m gpu suite and smoke() at the round's last code
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4final}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
