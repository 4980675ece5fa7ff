# round 5, pass 33: pinned host<->device copy rates by stream count
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bc}
mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/pcie_probe.py > $O/pcie.jsonl 2> $O/pcie.err || { echo "PROBE FAILED"; tail -20 $O/pcie.err; exit 1; }
cat $O/pcie.jsonl
