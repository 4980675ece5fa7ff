# round 5, pass 9: the crypter API GPU tests (striped list aggregate with out-of-range ciphertexts) and
# distributed.py's RCCL branches at world size 2 with both ranks on cuda:0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5n}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_crypter_api.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_crypter.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_crypter.txt; exit 1; }
tail -2 $O/pytest_crypter.txt
timeout -k 10 180 python -u tools/rccl_world2_probe.py --timeout 120 > $O/rccl_world2_probe.txt 2>&1 || { echo "RCCL PROBE FAILED"; tail -30 $O/rccl_world2_probe.txt; exit 1; }
tail -1 $O/rccl_world2_probe.txt
