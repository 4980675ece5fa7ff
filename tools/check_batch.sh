#!/bin/bash
# Batched-exponentiation check: its GPU tests, the whole GPU suite, then the bench at 10M and at the
# 1/8 stripe with and without the batch (A/B, each run under its own limit).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-batch}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_exp_batch.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_batch.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit 1
for rep in 1 2; do
  for n in 1250010 10000000; do
    for b in "" "--no-batch-exp"; do
      timeout -k 10 300 python -u bench.py --elements $n --steps 3 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e --no-stages $b > $O/b_${n}${b}_$rep.json 2> $O/b_${n}${b}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/b_${n}${b}_$rep.json').read().strip().splitlines()[-1]); print('n=$n $b', round(d['ms_per_step'],2), 'ms/step', round(d['value']/1e6,3), 'M/s')"
    done
  done
done
