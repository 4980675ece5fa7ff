# round 4: the triple engine's quotient broadcasts on the VALU (two DPP adds over a lane-masked digit,
# FBM_GEN_TRI_DPP=1 -> build/ab/tridpp.so, tools/ab_gen_variant.py) against the shipped ds_bpermute
# broadcasts (base4 = a copy of the shipped library): the group-engine GPU parity tests on the variant,
# then triple launches at one rank's 1/8 and 1/4 stripe, interleaved; then the multi-rank bench
# rehearsal of the shipped library (bench.py --gpus 2, gloo, one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4dpp}
mkdir -p $O
lib() { echo $GRAFT_REPO_ROOT/build/ab/$1.so; }
FBM_LIB_PATH=$(lib tridpp) timeout -k 10 400 python -u -m pytest tests/test_quad_engine.py tests/test_exp_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_tridpp.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_tridpp.txt; exit 1; }
tail -2 $O/pytest_tridpp.txt
for rep in 1 2 3; do
  for v in base4 tridpp; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 41667,83334 --engines triple --reps 3 > $O/probe_tri_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED tri $v"; tail -3 $O/probe_tri_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_tri_$v.$rep.jsonl
  done
done
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --elements 2000000 --steps 2 --warmup 1 > $O/dist2.json 2> $O/dist2.err || { rc=$?; echo "dist2 rc=$rc"; tail -c 1500 $O/dist2.err; exit $rc; }
tail -c 400 $O/dist2.json; echo
