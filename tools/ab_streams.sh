#!/bin/bash
# JL step time against the number of HIP streams the parties' encrypts use (one box,
# interleaved twice): bash tools/ab_streams.sh <outdir> "<counts>"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for rep in 1 2; do
  for k in $2; do
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e --streams $k \
      > $O/s$k.$rep.json 2> $O/s$k.$rep.err || { echo "FAIL $k"; tail -5 $O/s$k.$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('streams', sys.argv[2], 'value %.4g' % d['value'], 'ms/step %.1f' % d['ms_per_step'])" $O/s$k.$rep.json $k
  done
done
