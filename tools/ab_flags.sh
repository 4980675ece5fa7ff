#!/bin/bash
# JL bench A/B over flag sets on one box, interleaved twice:
#   bash tools/ab_flags.sh <outdir> "<flags A>" "<flags B>" ...   ("-" = no extra flags)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd $R
for rep in 1 2; do
  i=0
  for f in "$@"; do
    i=$((i + 1))
    [ "$f" = "-" ] && f=""
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e $f \
      > $O/v$i.$rep.json 2> $O/v$i.$rep.err || { echo "FAIL $f"; tail -5 $O/v$i.$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('[%s]' % sys.argv[2], 'value %.4g' % d['value'], 'ms/step %.1f' % d['ms_per_step'], 'exp/launch %.1f' % d['roofline']['avg_launch_ms'])" $O/v$i.$rep.json "$f"
  done
done
