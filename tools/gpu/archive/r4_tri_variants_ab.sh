# round 4: triple-engine variants (build/ab/<name>.so from tools/ab_gen_variant.py under FBM_GEN_* switches)
# against base4 (a copy of the shipped library): the group-engine GPU parity tests on every variant, then
# triple launches at one rank's 1/8 and 1/4 stripe, interleaved.   usage: r4_tri_variants_ab.sh OUT v1 v2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
lib() { echo $GRAFT_REPO_ROOT/build/ab/$1.so; }
for v in "$@"; do
  FBM_LIB_PATH=$(lib $v) timeout -k 10 400 python -u -m pytest tests/test_quad_engine.py tests/test_exp_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.txt 2>&1 || { echo "PYTEST FAILED $v"; tail -40 $O/pytest_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.txt)"
done
for rep in 1 2 3; do
  for v in ${BASE:-base4} "$@"; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 41667,83334 --engines triple --reps 3 > $O/probe_tri_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED tri $v"; tail -3 $O/probe_tri_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep $(grep -h triple_ms $O/probe_tri_$v.$rep.jsonl | tr '\n' ' ')"
  done
done
