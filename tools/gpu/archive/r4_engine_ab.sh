# round 4: the one-lane engine's K' fold, trimmed mid-product reduction, h in registers, C broadcast and
# nude read in place (new = the shipped library) against HEAD's engine (base = build/ab/base.so):
# the -m gpu suite on the new library, then one-lane launches and the bench step of both, interleaved,
# then the new library's HBM-traffic passes (FETCH_SIZE / WRITE_SIZE) of one serialised step.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
lib() { case $1 in new) echo $GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so;; *) echo $GRAFT_REPO_ROOT/build/ab/$1.so;; esac; }
for rep in 1 2; do
  for v in base new; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072,262144 --engines single --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_$v.$rep.jsonl; exit 1; }
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 41667,83334 --engines triple --reps 3 > $O/probe_tri_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED tri $v"; tail -3 $O/probe_tri_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl $O/probe_tri_$v.$rep.jsonl
  done
done
for rep in 1 2; do
  for v in base new; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || { echo "BENCH FAILED $v"; tail -5 $O/bench_$v.$rep.err; exit 1; }
    echo "== bench $v $rep"; python -c "import json; d=json.load(open('$O/bench_$v.$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_valu']['peak_provenance']['gfx_clock_during_launch'].get('median_mhz'), d['stages']['agg_scaling_probe']['ratio_whole_over_stripe'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $GRAFT_REPO_ROOT/$O/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $GRAFT_REPO_ROOT/$O/pmc_write.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err
rc=$?
echo "pmc rc=$rc"
exit $rc
