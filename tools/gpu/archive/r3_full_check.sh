# round 3: the full -m gpu suite and smoke on the current library, then the one-lane engine's
# square priced without its non-multiply instructions (build/ab/nadic_madsonly.so, garbage results)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/r3b/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r3b/pytest_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/r3b/smoke.txt; exit 1; }
tail -2 gpurun_out/r3b/smoke.txt
for rep in 1 2; do
  for v in rot nadic_madsonly; do
    FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072,262144 --engines single --reps 2 > gpurun_out/r3b/nadic_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; exit 1; }
    echo "== $v $rep"; grep ct gpurun_out/r3b/nadic_$v.$rep.jsonl
  done
done
