# round 5, pass 12: the prepared list aggregate's timeline -- fine stripes of 32 768 ciphertexts (the
# default), none (the prepared one-lane-round stripes), 65 536 -- and the unprepared one
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5t}
mkdir -p $O
cd $R
for f in 32768 131072 65536; do
  FBM_FINE_STRIPE_CT=$f timeout -k 10 300 python -u tools/list_agg_trace.py --prepared --top 15 > $O/trace_prepared_$f.txt 2>&1 || { echo "TRACE $f FAILED"; tail -20 $O/trace_prepared_$f.txt; exit 1; }
  tail -1 $O/trace_prepared_$f.txt | cut -c1-400
done
timeout -k 10 300 python -u tools/list_agg_trace.py --top 15 > $O/trace_plain.txt 2>&1 || { echo "TRACE PLAIN FAILED"; exit 1; }
tail -1 $O/trace_plain.txt | cut -c1-400
