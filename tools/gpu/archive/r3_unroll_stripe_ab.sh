# round 3: the unrolled vs looped one-lane square on one rank's 1/8 stripe step (2.86 one-lane rounds in the
# batched launch) and on the 10M step, interleaved on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/unroll_stripe
mkdir -p $O
lib() { case $1 in new) echo $GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so;; *) echo $GRAFT_REPO_ROOT/build/ab/$1.so;; esac; }
for rep in 1 2; do
  for v in looped new; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u bench.py --elements 1250010 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra --no-stages > $O/stripe_$v.$rep.json 2> $O/stripe_$v.$rep.err || { echo "BENCH FAILED $v"; tail -5 $O/stripe_$v.$rep.err; exit 1; }
    echo "== stripe $v $rep"; python -c "import json; d=json.load(open('$O/stripe_$v.$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_valu']['peak_provenance']['gfx_clock_during_launch'].get('median_mhz'))"
  done
done
for v in looped new; do
  FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 196608,300000,375003 --engines single --reps 2 > $O/probe_$v.jsonl 2>&1 || { echo "PROBE FAILED $v"; exit 1; }
  echo "== $v"; grep ct $O/probe_$v.jsonl
done
