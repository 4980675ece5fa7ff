# round 5, pass 36: is the 1/8-stripe aggregate slower at HEAD than at the session's start? the two libraries
# (build/ab/r5start.so from e49d827's sources, build/ab/head.so), interleaved, the aggregate at N = 1 and 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bk}
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for v in r5start head; do
    FBM_AB_VARIANT=1 FBM_LIB_PATH=$R/build/ab/$v.so timeout -k 10 200 python -u tools/agg_breakdown.py --splits 1,8 --reps 5 > $O/$v.$rep.jsonl 2> $O/$v.$rep.err || { echo "FAIL $v"; tail -5 $O/$v.$rep.err; exit 1; }
    echo "$v rep $rep: $(grep -o '"split": [0-9]*, [^}]*wall_ms_median": [0-9.]*' $O/$v.$rep.jsonl | sed 's/"elements.*"wall_ms_median"/ median/' | tr '\n' ' ')"
  done
done
