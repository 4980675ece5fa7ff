# round 4: which of the launch-bytes changes costs the one-lane launch its ~1 %: the library before them
# (r4a), the shipped one (new), the shipped one with whole H rows (FBM_COMPACT_H=0: nude digit 1 only), and
# the shipped one with both nude digits stored (build/ab/nude72.so: compact H only).  Interleaved, one box:
# one-lane decryption-factor launches (no nude) at one and two chip rounds, then the bench step.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4tr2}
mkdir -p $O
run() {  # variant tag, library, extra env
  local v=$1 lib=$2 env=$3
  env FBM_LIB_PATH=$lib $env timeout -k 10 200 python -u tools/exp_probe.py --ct 131072,262144 --engines single --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_$v.$rep.jsonl; return 1; }
  env FBM_LIB_PATH=$lib $env timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || { echo "BENCH FAILED $v"; tail -5 $O/bench_$v.$rep.err; return 1; }
  echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl; python -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print(d['value'], d['roofline']['avg_launch_ms'], d['roofline_valu']['peak_provenance']['gfx_clock_during_launch'].get('median_mhz'), round(d['stages']['T_agg_ms'],2), round(d['stages']['T_enc_ms'],1))"
}
NEW=$GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so
for rep in 1 2; do
  run r4a $GRAFT_REPO_ROOT/build/ab/r4a.so "" || exit 1
  run new $NEW "" || exit 1
  run hfull $NEW "FBM_COMPACT_H=0" || exit 1
  run nude72 $GRAFT_REPO_ROOT/build/ab/nude72.so "" || exit 1
done
