#!/bin/bash
# Aggregate-side kernels at the full vector and at the 1/8 stripe: kernel trace + the
# FETCH_SIZE / WRITE_SIZE passes (default policies), after the parity tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmcagg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_jls_api.py $R/tests/test_crypter_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { echo pytest failed; exit 1; }
cd /tmp && export TMPDIR=/tmp
A="--steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages"
for n in 10000000 1250010; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $R/bench.py $A --elements $n > $O/bench_$n.json 2> $O/kt_$n.err || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$n -o run -- python3 $R/bench.py $A --elements $n > /dev/null 2> $O/fetch_$n.err || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$n -o run -- python3 $R/bench.py $A --elements $n > /dev/null 2> $O/write_$n.err || exit 1
done
echo done
