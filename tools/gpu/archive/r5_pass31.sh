# round 5, pass 31: where a small list-API call's time goes (config 1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ba}
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/small_call_probe.py > $O/small_call.jsonl 2> $O/small_call.err || { echo "PROBE FAILED"; tail -20 $O/small_call.err; exit 1; }
cat $O/small_call.jsonl
