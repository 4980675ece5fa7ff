# round 3: the group engines' short path (quad / triple: binary chain with the short-base product) --
# the full -m gpu suite, then engine launch times and the bench line (with the aggregate-scaling curve)
# against the table-path build (build/ab/base.so = the commit before the one-lane short path)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/shortg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
for rep in 1 2; do
  for v in base new; do
    L=$GRAFT_REPO_ROOT/build/ab/base.so
    [ $v = new ] && L=$GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so
    FBM_LIB_PATH=$L timeout -k 10 200 python -u tools/exp_probe.py --ct 21504,41667,83334 --engines triple,quad --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl
  done
done
for v in base new; do
  L=$GRAFT_REPO_ROOT/build/ab/base.so
  [ $v = new ] && L=$GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so
  FBM_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra > $O/bench_$v.json 2> $O/bench_$v.err || { echo "BENCH FAILED $v"; tail -5 $O/bench_$v.err; exit 1; }
  echo "== bench $v"; python -c "import json; d=json.load(open('$O/bench_$v.json')); print(d['value'], d['ms_per_step'], d['stages']['T_agg_ms'], {k: round(v['T_agg_stripe_ms'],2) for k, v in d['stages']['agg_scaling_probe']['curve'].items()}, {k: round(v['ratio_whole_over_stripe'],3) for k, v in d['stages']['agg_scaling_probe']['curve'].items()})"
done
