# round 5, pass 27: both fuzz files with the prepared paths
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5au}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_fuzz_jls.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_fuzz.txt 2>&1 || { echo "FUZZ FAILED"; grep -E "FAILED|Error|assert" $O/pytest_fuzz.txt | head -30; exit 1; }
tail -1 $O/pytest_fuzz.txt
