#!/bin/bash
# A/B of GPU_MAX_HW_QUEUES (HIP's hardware queues per process, default 4) on the bench step:
# the parties' per-stream launches share FIFO hardware queues, so with 4 queues at most 4 of
# the P + 1 exponentiations run concurrently.  Each run under its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-hwq}
mkdir -p $O
cd $R
for q in 4 8 16 4 8 16; do
  for n in 1250010 10000000; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --elements $n --steps 3 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > $O/q${q}_n${n}.json 2> $O/q${q}_n${n}.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$O/q${q}_n${n}.json').read().strip().splitlines()[-1]); print('q=$q n=$n', round(d['ms_per_step'],2), 'ms/step', round(d['value']/1e6,3), 'M/s')"
  done
done
