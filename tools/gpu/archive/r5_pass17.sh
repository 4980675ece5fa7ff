# round 5, pass 17: the plain-C client of the C ABI (tests/c_client) against the oracle on the GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ai}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_c_client.py tests/test_host_conv.py -v --timeout 200 --timeout-method thread > $O/pytest_c_client.txt 2>&1 || { echo "C CLIENT FAILED"; grep -E "FAILED|Error|assert|fbm_c_roundtrip" $O/pytest_c_client.txt | head -30; exit 1; }
tail -2 $O/pytest_c_client.txt
