# round 4: one node's list-API encrypt at 10M elements -- stripe arrival / conversion timestamps, then the
# same under a kernel + memory-copy trace (are the stripes' device-to-host copies SDMA or blit kernels
# queued behind the next stripe's exponentiation?).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4node}
mkdir -p $O
cd $R
for rep in 1 2; do
  for side in "" "--side"; do
    timeout -k 10 300 python -u tools/node_encrypt_probe.py --reps 3 $side >> $O/node_probe.jsonl 2>> $O/node_probe.err || { echo "PROBE FAILED"; tail -20 $O/node_probe.err; exit 1; }
  done
done
cat $O/node_probe.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/node_encrypt_probe.py --reps 1 --side > $O/node_probe_traced.jsonl 2> $O/trace.err
rc=$?
echo "trace rc=$rc"
exit $rc
