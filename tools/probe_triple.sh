#!/bin/bash
# Triple-engine check on the GPU box: the engine equivalence tests first (bit-exact vs the one-lane
# engine and the oracle), then the full GPU suite, then the exponentiation sweep over launch sizes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-triple}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_quad_engine.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_engines.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
timeout -k 10 300 python -u tools/exp_probe.py --engines single,quad,triple --ct 16384,21504,32768,41667,43008,49152,64512 --reps 2 > $O/occ.jsonl 2> $O/occ.err &&
timeout -k 10 200 python -u tools/agg_scaling.py > $O/agg_scaling.json 2> $O/agg_scaling.err
rc=$?; echo rc=$rc; tail -3 $O/pytest_engines.txt $O/pytest_gpu.txt; cat $O/occ.jsonl $O/agg_scaling.json; exit $rc
