# round 5: LOM aggregate variants (tools/microbench/agg_variants.hip) at config-5 and bench shapes, and the
# int8-MFMA Montgomery-reduction pricing kernel (tools/microbench/mfma_redc.hip), built in-tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5c}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/microbench/mfma_redc_check.py --ct 131072 --iters 64 --reps 5 --check 256 > $O/mfma_redc.json 2>&1 || { echo "MFMA REDC FAILED"; cat $O/mfma_redc.json; exit 1; }
cat $O/mfma_redc.json
timeout -k 10 300 python -u tools/microbench/mfma_redc_check.py --ct 262144 --iters 64 --reps 5 --check 64 > $O/mfma_redc_2r.json 2>&1 || { echo "MFMA REDC 2R FAILED"; cat $O/mfma_redc_2r.json; exit 1; }
cat $O/mfma_redc_2r.json
for PN in "16 100000000" "8 99999744" "16 9999872" "8 9999872"; do
  set -- $PN
  timeout -k 10 300 ./tools/microbench/agg_variants $2 $1 7 > $O/aggv_P$1_n$2.jsonl 2>&1 || { echo "AGG VARIANTS FAILED $PN"; tail -5 $O/aggv_P$1_n$2.jsonl; exit 1; }
  grep '"pass": 1' $O/aggv_P$1_n$2.jsonl
done
