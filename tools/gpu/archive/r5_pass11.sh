# round 5, pass 11: the N > 1 bench path rehearsed on one GPU at this round's code (gloo, 2 and 4 ranks),
# and the per-kernel breakdown of the aggregate on rank 0's stripe of a 1/2/4/8-GPU split
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5s}
mkdir -p $O
cd $R
python -c "import os; from fedbiomed_amd import _device as D; print(\"cgroup quota\", D.cgroup_cpu_quota(), \"affinity\", len(os.sched_getaffinity(0)))"
timeout -k 10 300 python -u -m pytest tests/test_crypter_api.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_crypter.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_crypter.txt; exit 1; }
tail -2 $O/pytest_crypter.txt
bash tools/rehearse_dist.sh ${1:-r5s} || exit 1
timeout -k 10 300 python -u tools/agg_breakdown.py > $O/agg_breakdown.jsonl 2> $O/agg_breakdown.err || { echo "AGG BREAKDOWN FAILED"; tail -20 $O/agg_breakdown.err; exit 1; }
tail -3 $O/agg_breakdown.jsonl
timeout -k 10 300 python -u tools/list_agg_probe.py --first-call plain > $O/first_call_plain.jsonl 2>&1 || { echo "FIRST CALL PLAIN FAILED"; tail -5 $O/first_call_plain.jsonl; exit 1; }
tail -1 $O/first_call_plain.jsonl
timeout -k 10 300 python -u tools/list_agg_probe.py --first-call prepared > $O/first_call_prepared.jsonl 2>&1 || { echo "FIRST CALL PREPARED FAILED"; tail -5 $O/first_call_prepared.jsonl; exit 1; }
tail -1 $O/first_call_prepared.jsonl
FBM_AGG_TAIL_SPLIT=0 timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8 > $O/list_agg_probe_nosplit.jsonl 2>&1 || { echo "PROBE NOSPLIT FAILED"; exit 1; }
tail -1 $O/list_agg_probe_nosplit.jsonl
timeout -k 10 300 python -u tools/list_agg_probe.py --threads 8 > $O/list_agg_probe.jsonl 2>&1 || { echo "PROBE FAILED"; exit 1; }
tail -1 $O/list_agg_probe.jsonl
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
