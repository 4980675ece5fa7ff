# round 5, pass 16: bytes_to_ints with its digits written on host threads; results freed outside the clock --
# (box CPUs), one node's 10M-element list encrypt, and the bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ah}
mkdir -p $O
cd $R
timeout -k 10 120 python -u tools/convbench.py 1 8 16 > $O/convbench.txt 2>&1 || { echo "CONVBENCH FAILED"; tail -20 $O/convbench.txt; exit 1; }
cat $O/convbench.txt
timeout -k 10 200 python -u tools/node_encrypt_probe.py --elements 10000000 --reps 4 > $O/node_probe.txt 2>&1 || { echo "NODE PROBE FAILED"; tail -20 $O/node_probe.txt; exit 1; }
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$O/bench.json')); e=d['end_to_end']; print(d['value'], json.dumps(e['node_encrypt_list_api']), e['list_api']['value'], e['lom']['list_api']['value'])"
