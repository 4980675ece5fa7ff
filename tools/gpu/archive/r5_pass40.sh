# round 5, pass 40: after the launch-shape change, auto's pick against every engine at the path's sizes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bp}
mkdir -p $O
cd $R
timeout -k 10 500 python -u tools/exp_probe.py --ct 33334,41667,62500,71190,83334,100000 --engines single,triple,quad,auto > $O/engines.jsonl 2> $O/engines.err || { echo "PROBE FAILED"; tail -5 $O/engines.err; exit 1; }
cut -c1-220 $O/engines.jsonl
