# round 3: the triple engine's row parts priced inside the real launch (garbage results)
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in rot tri_noret64 tri_nochain tri_madsonly; do
    FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 200 python -u tools/exp_probe.py --ct 21504,43008,86016 --engines triple --reps 3 > gpurun_out/trireal_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 gpurun_out/trireal_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct gpurun_out/trireal_$v.$rep.jsonl
  done
done
