# round 4: one-lane engine variants (build/ab/<name>.so, tools/ab_gen_variant.py under FBM_GEN_* switches)
# against ${BASE:-cur} (a copy of the shipped library): the JL GPU parity tests on every variant, one-lane
# launches at a lone wave / one round / two rounds per SIMD, then the 10M x 8 bench step, interleaved.
#   usage: r4_single_ab.sh OUT v1 v2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
B=${BASE:-cur}
lib() { echo $GRAFT_REPO_ROOT/build/ab/$1.so; }
for v in "$@"; do
  FBM_LIB_PATH=$(lib $v) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_exp_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.txt 2>&1 || { echo "PYTEST FAILED $v"; tail -40 $O/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.txt)"
done
for rep in 1 2; do
  for v in $B "$@"; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072,262144 --engines single --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep $(grep -h _ms $O/probe_$v.$rep.jsonl | tr '\n' ' ')"
  done
done
for rep in 1 2; do
  for v in $B "$@"; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || { echo "BENCH FAILED $v"; tail -5 $O/bench_$v.$rep.err; exit 1; }
    echo "== bench $v $rep $(python -c "import json; d=json.loads([l for l in open('$O/bench_$v.$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['ms_per_step'],1), d['roofline_valu']['peak_provenance']['gfx_clock_during_launch'].get('median_mhz'), round(d['stages']['agg_scaling_probe']['ratio_whole_over_stripe'],3))")"
  done
done
