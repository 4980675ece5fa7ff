# round 3: rotated mad carry-outs -- engine parity on the new library, then A/B of the engines'
# launch times and of the bench step against the vcc-only build (build/ab/{vcc,rot}.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_quad_engine.py tests/test_exp_batch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/rot_tests.log 2>&1 || { echo "TESTS FAILED"; tail -20 gpurun_out/rot_tests.log; exit 1; }
tail -2 gpurun_out/rot_tests.log
for rep in 1 2; do
  for v in vcc rot; do
    FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 200 python -u tools/exp_probe.py --ct 41667,83334,333334 --engines single,triple,quad --reps 3 > gpurun_out/rot_probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -5 gpurun_out/rot_probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; cat gpurun_out/rot_probe_$v.$rep.jsonl | grep ct
  done
done
for v in vcc rot; do
  FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra > gpurun_out/rot_bench_$v.json 2> gpurun_out/rot_bench_$v.err || { echo "BENCH FAILED $v"; tail -5 gpurun_out/rot_bench_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('stages',{}).get('agg_scaling_probe',{}).get('curve'))" gpurun_out/rot_bench_$v.json $v
done
