# round 5, pass 41: the LOM host-buffer one-call path (ABI 6) -- its tests, the LOM / ABI GPU tests, the
# small-call probe and BASELINE configs 1-3 through the list API
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5br}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_lom_host_call.py tests/test_native_abi.py tests/test_capi_validation.py tests/test_c_client.py \
  tests/test_gpu_parity.py tests/test_crypter_api.py tests/test_crypter_sweep.py tests/test_exceptions_bound.py \
  tests/test_edge_weights.py tests/test_configs.py tests/test_caller_flows.py tests/test_encrypt_factor.py \
  > $O/pytest.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|passed|failed" $O/pytest.log | tail -30; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -u tools/small_call_probe.py --reps 300 > $O/small_call.jsonl 2> $O/small_call.err || { echo "PROBE FAILED"; tail -5 $O/small_call.err; exit 1; }
cat $O/small_call.jsonl
timeout -k 10 300 python -u tools/bench_configs.py --reps 5 > $O/bench_configs.jsonl 2> $O/bench_configs.err || { echo "CONFIGS FAILED"; tail -5 $O/bench_configs.err; exit 1; }
cut -c1-400 $O/bench_configs.jsonl
