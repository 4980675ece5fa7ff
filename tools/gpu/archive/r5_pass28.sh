# round 5, pass 28: additive shares from the reference's stream -- the ASS tests on the GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5av}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ass.py tests/test_host_conv.py tests/test_caller_flows.py -v --timeout 200 --timeout-method thread > $O/pytest_ass.txt 2>&1 || { echo "ASS FAILED"; grep -E "FAILED|Error|assert" $O/pytest_ass.txt | head -30; exit 1; }
tail -1 $O/pytest_ass.txt
