# round 4 baseline on a fresh box: the -m gpu suite at HEAD, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4base
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_valu']['peak_provenance']['gfx_clock_during_launch'].get('median_mhz'))"
