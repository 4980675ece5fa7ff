# round 5, pass 15: the seeded random list-API cases of both crypters against the oracle
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ac}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_fuzz_jls.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_fuzz.txt 2>&1 || { echo "FUZZ FAILED"; grep -E "FAILED|Error|assert" $O/pytest_fuzz.txt | head -30; exit 1; }
tail -2 $O/pytest_fuzz.txt
