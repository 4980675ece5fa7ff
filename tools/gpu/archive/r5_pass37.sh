# round 5, pass 37: the group engines' workgroup placement -- the aggregate's 1/8 and 1/4 stripes with the
# launch capped at two workgroups per CU by dynamic LDS (FBM_GROUP_LDS_PAD=26624) against the default, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bl}
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for pad in 0 26624; do
    FBM_GROUP_LDS_PAD=$pad timeout -k 10 200 python -u tools/agg_breakdown.py --splits 8,4 --reps 7 > $O/pad$pad.$rep.jsonl 2> $O/pad$pad.$rep.err || { echo "FAIL $pad"; tail -5 $O/pad$pad.$rep.err; exit 1; }
    echo "pad $pad rep $rep: $(grep -o '"split": [0-9]*, [^}]*wall_ms_median": [0-9.]*' $O/pad$pad.$rep.jsonl | sed 's/"elements.*"wall_ms_median"/ median/' | tr '\n' ' ')"
  done
done
