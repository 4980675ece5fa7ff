# round 5, pass 34: the prepared list aggregate's pipelining stripes (FBM_PREP_STRIPE_CT) at 10M x 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bd}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_crypter_api.py -m gpu -k prepare -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "TEST FAILED"; grep -E "FAILED|Error|assert" $O/pytest.txt | head; exit 1; }
tail -1 $O/pytest.txt
for s in 131072 65536 32768 16384; do  # (FBM_PREP_STRIPE_CT: the reverted finer-stripes change, b31fcd4)
  FBM_PREP_STRIPE_CT=$s timeout -k 10 300 python -u tools/list_agg_probe.py --threads 16 --prepare-each > $O/prep_$s.jsonl 2>&1 || { echo "PROBE $s FAILED"; tail -20 $O/prep_$s.jsonl; exit 1; }
  echo "stripe_ct=$s $(grep conv_threads $O/prep_$s.jsonl | cut -c1-200)"
done
