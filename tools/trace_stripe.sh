R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace_stripe
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 $R/bench.py --elements 1250010 --steps 2 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > $O/b.json 2> $O/b.err
rc=$?; echo rc=$rc; tail -c 300 $O/b.json; exit $rc
