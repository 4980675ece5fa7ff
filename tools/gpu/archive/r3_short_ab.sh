# round 3: the one-lane engine's short path (binary chain over |key| with the short-base product,
# no window table) -- the full -m gpu suite on the new library, then launch times and the bench
# step against the table-path build of the previous commit (build/ab/base.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/short
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
for rep in 1 2; do
  for v in base new; do
    L=$GRAFT_REPO_ROOT/build/ab/base.so
    [ $v = new ] && L=$GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so
    FBM_LIB_PATH=$L timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072,262144 --engines single --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl
  done
done
for v in base new; do
  L=$GRAFT_REPO_ROOT/build/ab/base.so
  [ $v = new ] && L=$GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so
  FBM_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra > $O/bench_$v.json 2> $O/bench_$v.err || { echo "BENCH FAILED $v"; tail -5 $O/bench_$v.err; exit 1; }
  echo "== bench $v"; cut -c1-220 $O/bench_$v.json
done
