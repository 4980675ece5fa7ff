# round 5, pass 20: the encrypt with its factor computed ahead (fbm_jl_encrypt_factor, prepare_encrypt)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5am}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_encrypt_factor.py tests/test_c_client.py tests/test_native_abi.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_encf.txt 2>&1 || { echo "ENCF FAILED"; grep -E "FAILED|Error|assert" $O/pytest_encf.txt | head -30; exit 1; }
tail -2 $O/pytest_encf.txt
