# round 5, pass 4: the -m gpu suite (ABI 4: signed VES, wide FDH), config 5's trace + HBM-traffic passes
# with the wave-split kernels, and the one-GPU strong-scaling prediction
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5g}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
bash tools/gpu/r5_pass3.sh ${1:-r5g}
cd $R && timeout -k 10 300 python -u tools/list_agg_probe.py --threads 4,8,16 > $O/list_agg_probe.jsonl 2>&1 || { echo "LIST AGG PROBE FAILED"; tail -5 $O/list_agg_probe.jsonl; exit 1; }
cat $O/list_agg_probe.jsonl
