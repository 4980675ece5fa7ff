# round 5, pass 19: the host conversions' default thread count from the process's CPU share -- bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ak}
mkdir -p $O
cd $R
python -c "from fedbiomed_amd import _device as D; print('cpu share', D.host_cpu_share(), 'quota', D.cgroup_cpu_quota())"
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); e=d['end_to_end']; r=e['researcher_aggregate_list_api']; print(d['value'], json.dumps(r['at_metric_size']), json.dumps(e['node_encrypt_list_api']['10000000']), e['list_api']['value'], e['lom']['list_api']['value'])"
