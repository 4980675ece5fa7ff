# round 5, pass 35: the C ABI's argument refusals
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bi}
mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest tests/test_capi_validation.py tests/test_wire.py -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/pytest.txt | head -30; exit 1; }
tail -1 $O/pytest.txt
