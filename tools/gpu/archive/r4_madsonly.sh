# round 4: the shipped engines' squares priced without their non-multiply instructions, inside the real launch
# (tools/ab_engine_variants.py: build/ab/{nadic,tri}_madsonly.so -- garbage results, timing only) against the
# shipped library (build/ab/cur.so, a copy): one-lane launches at a lone wave / one round / two rounds per SIMD,
# triple at one rank's 1/8 and 1/4 stripe, two interleaved passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4mo}
mkdir -p $O
lib() { echo $GRAFT_REPO_ROOT/build/ab/$1.so; }
for rep in 1 2; do
  for v in cur nadic_madsonly; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072,262144 --engines single --reps 2 > $O/probe_single_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_single_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep $(grep -h _ms $O/probe_single_$v.$rep.jsonl | tr '\n' ' ')"
  done
  for v in cur tri_madsonly; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 41667,83334 --engines triple --reps 3 > $O/probe_tri_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED tri $v"; tail -3 $O/probe_tri_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep $(grep -h _ms $O/probe_tri_$v.$rep.jsonl | tr '\n' ' ')"
  done
done
