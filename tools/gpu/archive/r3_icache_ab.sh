# round 3: is the unrolled square's 375k-ciphertext slowdown the launch's code size?  Three builds of the
# one-lane kernel interleaved on one box: looped (build/ab/looped.so: looped square everywhere), new (the
# unrolled square on the short path only, 167 KB kernel), shortonly (build/ab/shortonly.so: no table path,
# 106 KB); decryption-factor launches at 2.29 / 2.86 / 4 rounds and the 1/8-stripe step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/icache
mkdir -p $O
lib() { case $1 in new) echo $GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so;; *) echo $GRAFT_REPO_ROOT/build/ab/$1.so;; esac; }
for rep in 1 2; do
  for v in looped new shortonly; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 300000,375003,524288 --engines single --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl
  done
done
for v in looped new shortonly; do
  FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u bench.py --elements 1250010 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra --no-stages > $O/stripe_$v.json 2> $O/stripe_$v.err || { echo "BENCH FAILED $v"; tail -5 $O/stripe_$v.err; exit 1; }
  echo "== stripe $v"; python -c "import json; d=json.load(open('$O/stripe_$v.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_valu']['peak_provenance']['gfx_clock_during_launch'].get('median_mhz'))"
done
