#!/bin/bash
# SQ counter passes over the exponentiation alone (tools/exp_probe.py), one process per pass
# under a hard time limit; the chain stops at the first failure.  Usage: tools/pmc_exp.sh TAG [probe args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmc_exp}
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/exp_probe.py "$@" > $O/trace.json 2> $O/trace.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc1 -o run -- python3 $R/tools/exp_probe.py "$@" > $O/pmc1.json 2> $O/pmc1.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $O/pmc2 -o run -- python3 $R/tools/exp_probe.py "$@" > $O/pmc2.json 2> $O/pmc2.err
rc=$?
echo "rc=$rc"; tail -2 $O/trace.err $O/pmc1.err $O/pmc2.err; cat $O/trace.json
exit $rc
