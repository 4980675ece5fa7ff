# round 5, pass 2: the MFMA-reduction pricing kernel, the aggregate variants, then the library with the
# wave-split LOM aggregate / ASS reconstruct: the -m gpu suite, config 5 and the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5e}
mkdir -p $O
cd $R
bash tools/gpu/r5_aggv.sh ${1:-r5e} || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -u tools/bench_cfg5.py > $O/cfg5_bench.json 2> $O/cfg5_bench.err || { echo "CFG5 FAILED"; tail -5 $O/cfg5_bench.err; exit 1; }
cat $O/cfg5_bench.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
