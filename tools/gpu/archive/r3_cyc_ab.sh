# round 3: the cyclic-band triangular square of the group engines -- parity through every engine
# on the new library, then launch times against the previous build (build/ab/{rot,cyc}.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_quad_engine.py tests/test_exp_batch.py tests/test_gpu_parity.py tests/test_even_moduli.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/cyc_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/cyc_tests.log; exit 1; }
tail -2 gpurun_out/cyc_tests.log
for rep in 1 2; do
  for v in rot cyc; do
    FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 200 python -u tools/exp_probe.py --ct 21504,41667,83334 --engines triple,quad --reps 3 > gpurun_out/cyc_probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 gpurun_out/cyc_probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct gpurun_out/cyc_probe_$v.$rep.jsonl
  done
done
