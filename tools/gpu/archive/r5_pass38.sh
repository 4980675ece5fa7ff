# round 5, pass 38: group-engine workgroups launched per CU (FBM_GROUP_WGS 2 vs 3), the aggregate's stripes at
# N = 8 / 4 and the triple / quad launch sweep between, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bm}
mkdir -p $O
cd $R
for rep in 1 2; do
  for w in 3 2; do
    FBM_GROUP_WGS=$w timeout -k 10 200 python -u tools/agg_breakdown.py --splits 8,4 --reps 7 > $O/w$w.$rep.jsonl 2> $O/w$w.$rep.err || { echo "FAIL $w"; tail -5 $O/w$w.$rep.err; exit 1; }
    echo "wgs $w rep $rep: $(grep -o '"split": [0-9]*, [^}]*wall_ms_median": [0-9.]*' $O/w$w.$rep.jsonl | sed 's/"elements.*"wall_ms_median"/ median/' | tr '\n' ' ')"
  done
done
for w in 3 2; do
  FBM_GROUP_WGS=$w timeout -k 10 300 python -u tools/exp_probe.py --ct 21504,32256,43008,55000,64512,75000,86016,100000 --engines triple,quad > $O/sweep_w$w.jsonl 2> $O/sweep_w$w.err || { echo "SWEEP FAIL $w"; tail -5 $O/sweep_w$w.err; exit 1; }
  echo "sweep wgs $w"; cut -c1-160 $O/sweep_w$w.jsonl
done
