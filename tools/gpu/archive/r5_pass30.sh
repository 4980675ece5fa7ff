# round 5, pass 30: the unprepared list encrypt's ints made during the exponentiation -- parity tests, node probe, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ay}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_crypter_api.py tests/test_gpu_fuzz.py tests/test_encrypt_factor.py tests/test_caller_flows.py tests/test_configs.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/pytest.txt | head -30; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 200 python -u tools/node_encrypt_probe.py --elements 10000000 --reps 3 > $O/node_probe.txt 2>&1 || { echo "NODE PROBE FAILED"; tail -20 $O/node_probe.txt; exit 1; }
grep elements $O/node_probe.txt | cut -c1-400
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); e=d['end_to_end']; print(d['value'], json.dumps(e['node_encrypt_list_api']), e['list_api']['value'])"
