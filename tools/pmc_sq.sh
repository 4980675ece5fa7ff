#!/bin/bash
# SQ/GRBM counter pass over one serialised bench step (stall breakdown + effective clock).
# Each pass is its own process under a hard time limit; the chain stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sq}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc1 -o run -- python3 $R/bench.py $ARGS > $O/pmc1.json 2> $O/pmc1.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $O/pmc2 -o run -- python3 $R/bench.py $ARGS > $O/pmc2.json 2> $O/pmc2.err
rc=$?
echo "rc=$rc"; tail -3 $O/pmc1.err $O/pmc2.err
exit $rc
