#!/bin/bash
# Round check on the GPU box: GPU parity tests, smoke, default bench line, aggregate scaling probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-check}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python -u tools/agg_scaling.py > $O/agg_scaling.json 2> $O/agg_scaling.err
rc=$?
echo "rc=$rc"
tail -3 $O/pytest_gpu.txt
cat $O/smoke.txt $O/bench.json $O/agg_scaling.json
exit $rc
