#!/bin/bash
# Strong-scaling prediction on ONE GPU: the bench step on the largest stripe one rank owns in an
# N-GPU split of the 10M-element vector (N = 1, 2, 4, 8; distributed.shard_range, 30-element
# alignment).  Predicted value(N) = 10M / T_step(stripe); efficiency = T_step(10M) / (N T_step).
# Every GPU step has its own time limit; the chain stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-predict}
mkdir -p $O
cd $R
for n in 10000000 5000010 2500020 1250010; do
  timeout -k 10 240 python -u bench.py --elements $n --steps 5 --warmup 1 --no-cpu-baseline --no-lom-extra --no-e2e \
    > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
done
python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
rows = {}
for n, N in ((10000000, 1), (5000010, 2), (2500020, 4), (1250010, 8)):
    d = json.loads(open(f"{o}/bench_{n}.json").read().strip().splitlines()[-1])
    rows[N] = (n, d["ms_per_step"], d["stages"]["T_agg_ms"])
t1, a1 = rows[1][1], rows[1][2]
out = []
for N, (n, t, a) in rows.items():
    out.append({"n_gpus": N, "stripe_elements": n, "ms_per_step": t, "predicted_value": 10_000_000 / (t / 1000),
                "step_speedup": t1 / t, "efficiency": t1 / (N * t), "T_agg_ms": a, "agg_speedup": a1 / a})
json.dump(out, open(f"{o}/predicted_scaling.json", "w"), indent=1)
for r in out:
    print(json.dumps(r))
PY
