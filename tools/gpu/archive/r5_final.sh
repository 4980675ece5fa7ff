# round 5 final pass: the -m gpu suite, smoke(), the default bench line, and rocprofv3 --kernel-trace --stats
# of one serialised 10M step (the line's avg_launch_ms against the profiler's)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5o}
mkdir -p $O/jl
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/jl/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > $O/jl/prof_bench.json 2> $O/jl/prof.err
rc=$?
echo "rc=$rc"
exit $rc
