# round 4 measurement pass (run through gpurun from the repo root): the -m gpu suite and smoke, the
# default bench line (with the node list-API legs and the CPU baseline), the kernel trace + stats and
# the two HBM-traffic PMC passes of one serialised bench step, the 1/8 stripe bench, the MAD peak, and
# the generic engine at bench-like scale (odd modulus forced to generic, and an even modulus, which
# only the generic engine takes).  Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4m}
mkdir -p $O
cd $R
if [ -z "$SKIP_PYTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.txt; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --elements 1250010 --steps 5 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e > $O/bench_stripe8.json 2> $O/bench_stripe8.err || { echo "STRIPE8 FAILED"; exit 1; }
timeout -k 10 200 python -u tools/exp_probe.py --ct 16384 --engines generic --reps 2 > $O/generic_odd.jsonl 2>&1 || { echo "GENERIC FAILED"; tail -5 $O/generic_odd.jsonl; exit 1; }
timeout -k 10 200 python -u tools/exp_probe.py --ct 16384 --engines auto --reps 2 --even > $O/generic_even.jsonl 2>&1 || { echo "GENERIC EVEN FAILED"; tail -5 $O/generic_even.jsonl; exit 1; }
cat $O/generic_odd.jsonl $O/generic_even.jsonl
if [ -x ./tools/microbench/madpeak ]; then timeout -k 10 120 ./tools/microbench/madpeak 400000 > $O/madpeak.txt 2>&1 || exit 1; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > $O/prof_bench.json 2> $O/prof.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $O/pmc_fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $O/pmc_write.err
rc=$?
echo "rc=$rc"
exit $rc
