# round 5, pass 39: two group workgroups per CU by default -- the GPU suite (every engine's parity), the bench's probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5bn}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error|assert" $O/pytest_gpu.txt | head -30; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); p=d['stages']['agg_scaling_probe']; print(d['value'], d['stages']['T_agg_ms'], {k: (round(v['T_agg_stripe_ms'],2), round(v['ratio_whole_over_stripe'],3), round(v['ratio_with_gather'],3)) for k, v in p['curve'].items()})"
timeout -k 10 200 python -u tools/agg_breakdown.py --splits 1,2,4,8 --reps 5 > $O/agg_breakdown.jsonl 2> $O/agg_breakdown.err || { echo "BREAKDOWN FAILED"; tail -5 $O/agg_breakdown.err; exit 1; }
grep ratios $O/agg_breakdown.jsonl
