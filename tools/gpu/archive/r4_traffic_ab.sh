# round 4: the exponentiation launch's bytes -- compact H rows (32 B per ciphertext instead of 256; the whole
# row only behind a sentinel) and the nude operand's digit 1 only (144 B instead of 288; digit 0 as
# immediates, fbm_na_mm_nude) -- against the library before them (base = build/ab/r4a.so): the -m gpu
# suite on the new library, the bench step of both interleaved, then the new library's HBM-traffic passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4tr}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
lib() { case $1 in new) echo $GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so;; *) echo $GRAFT_REPO_ROOT/build/ab/$1.so;; esac; }
for rep in 1 2; do
  for v in r4a new; do
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
