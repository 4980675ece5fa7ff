set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -x -v --timeout 240 --timeout-method thread -m gpu -k "rccl" > gpurun_out/rccl.log 2>&1; echo "RCCL TEST EXIT $?"; tail -5 gpurun_out/rccl.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; echo "BENCH EXIT $?"; tail -c 600 gpurun_out/bench_default.err
timeout -k 10 300 python -u bench.py --rccl-world1 --steps 2 --no-cpu-baseline --no-e2e --no-lom-extra > gpurun_out/bench_rccl1.json 2> gpurun_out/bench_rccl1.err; echo "BENCH RCCL EXIT $?"; tail -c 600 gpurun_out/bench_rccl1.err
