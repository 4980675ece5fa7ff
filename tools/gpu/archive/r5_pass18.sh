# round 5, pass 18: the list aggregate at 10M x 8 by host-conversion thread count, plain and prepared
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5aj}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8,12,16 > $O/list_agg_plain.jsonl 2>&1 || { echo "PLAIN FAILED"; tail -20 $O/list_agg_plain.jsonl; exit 1; }
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8,12,16 --prepare-each > $O/list_agg_prepared.jsonl 2>&1 || { echo "PREPARED FAILED"; tail -20 $O/list_agg_prepared.jsonl; exit 1; }
grep conv_threads $O/list_agg_plain.jsonl $O/list_agg_prepared.jsonl
