# round 5, pass 23: the prepared encrypts' output pools (JL and LOM) -- tests and the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5aq}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_encrypt_factor.py tests/test_host_conv.py tests/test_prepare_cpu.py tests/test_lom_api.py tests/test_crypter_api.py -v --timeout 200 --timeout-method thread > $O/pytest_encf.txt 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/pytest_encf.txt | head -30; exit 1; }
tail -1 $O/pytest_encf.txt
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); e=d['end_to_end']; print(d['value'], json.dumps({k: v.get('factor_prepared') for k, v in e['node_encrypt_list_api'].items() if isinstance(v, dict)}), json.dumps(e['lom']['list_api']), json.dumps(e['lom']['node_encrypt_list_api']))"
