# round 5, pass 21: bench line with the node's prepared encrypt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5an}
mkdir -p $O
cd $R
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); e=d['end_to_end']; print(d['value'], json.dumps(e['node_encrypt_list_api']))"
