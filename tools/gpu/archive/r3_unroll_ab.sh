# round 3: the one-lane engine's square unrolled (no computed jumps / m0) vs looped, and the short product
# unrolled vs looped (code size: the unrolled square is 43 KB) -- the full -m gpu suite on the shipped library
# (unrolled square, looped short product), then one-lane launch times and the bench step of three builds:
#   looped = build/ab/looped.so (-DFBM_NA_LOOPED_SQUARE, unrolled short), unroll = build/ab/unroll.so
#   (both unrolled), new = the shipped library
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/unroll
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
lib() { case $1 in new) echo $GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so;; *) echo $GRAFT_REPO_ROOT/build/ab/$1.so;; esac; }
for rep in 1 2; do
  for v in looped unroll new; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072,262144 --engines single --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl
  done
done
for v in looped unroll new; do
  FBM_LIB_PATH=$(lib $v) timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-lom-extra --no-stages > $O/bench_$v.json 2> $O/bench_$v.err || { echo "BENCH FAILED $v"; tail -5 $O/bench_$v.err; exit 1; }
  echo "== bench $v"; python -c "import json; d=json.load(open('$O/bench_$v.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline_valu']['peak_provenance']['gfx_clock_during_launch'].get('median_mhz'))"
done
