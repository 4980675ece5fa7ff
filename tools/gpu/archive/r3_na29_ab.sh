# round 3: the one-lane engine at 29-bit limbs (36 per digit, mid-product reduction) -- the full
# -m gpu suite on the new library, then its launch times against the 28-bit build (build/ab/na28.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/na29
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/na29/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/na29/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/na29/pytest_gpu.txt
for rep in 1 2; do
  for v in na28 na29; do
    FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072,262144 --engines single --reps 2 > gpurun_out/na29/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 gpurun_out/na29/probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct gpurun_out/na29/probe_$v.$rep.jsonl
  done
done
for v in na28 na29; do
  FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 300 python -u bench.py > gpurun_out/na29/bench_$v.json 2> gpurun_out/na29/bench_$v.err || { echo "BENCH FAILED $v"; tail -5 gpurun_out/na29/bench_$v.err; exit 1; }
  echo "== bench $v"; cut -c1-200 gpurun_out/na29/bench_$v.json
done
