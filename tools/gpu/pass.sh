#!/bin/bash
# One parameterised measurement pass on the GPU box (run through gpurun from the repo root):
#
#   bash tools/gpu/pass.sh TAG STEP [STEP ...]
#
# Steps (each under its own time limit; the pass stops at the first failure and starts nothing
# more on the GPU):
#   tests      the -m gpu suite                               -> pytest_gpu.txt
#   smoke      __graft_entry__.smoke()                         -> smoke.txt
#   bench      the default bench line (the driver's command)   -> bench.json
#   jlprof     rocprofv3 --kernel-trace --stats of one serialised 10M x 8 JL step -> jl/prof
#   jlpmc      its FETCH_SIZE / WRITE_SIZE passes (separate runs)                 -> jl/pmc_*
#   lompmc     kernel trace + FETCH_SIZE / WRITE_SIZE of the LOM bench (10M x 8)  -> lom/...
#   dist8      bench.py --gpus 8 through spawn_ranks: 8 gloo ranks sharing this GPU, 2M elements
#   dist8full  the same at the metric's 10M elements and the driver's --steps 20 --warmup 5 (all 8 ranks'
#              work on one GPU: an upper bound on the driver's 8-GPU wall time)
#   dist8run   the driver's launch form: python -m torch.distributed.run --nproc-per-node 8 ... bench.py --gpus 8
#              (gloo instead of RCCL, which refuses eight ranks on one GPU), 2M elements
#   TEST=path  one test file / node id (e.g. TEST=tests/test_configs.py)
#   RUN=tools/x.py[,args]  a probe script (args comma-separated)         -> x.jsonl
# Summaries: python tools/prof_summary.py gpurun_out/TAG/jl profiles/TAG_jl (and .../lom).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PY="python -u"
JLARGS="--steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages"
LOMARGS="--scheme lom --steps 5 --warmup 1 --serial --no-cpu-baseline --no-e2e"

holders() {  # GPU processes left behind by a step (there should be none): polled for up to 15 s, since an
  local n w=0  # exited rank's GPU context can stay listed for a moment while the driver tears it down
  n=$(rocm-smi --showpids 2>/dev/null | grep -cE "^[0-9]+ " || true)
  while [ "$n" != "0" ] && [ $w -lt 15 ]; do
    sleep 1; w=$((w + 1))
    n=$(rocm-smi --showpids 2>/dev/null | grep -cE "^[0-9]+ " || true)
  done
  echo "gpu_holders_left: $n (after ${w} s)"
}

run_step() {
  local s=$1
  case $s in
  tests)
    timeout -k 10 900 $PY -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
    local rc=$?; tail -3 $O/pytest_gpu.txt; return $rc ;;
  TEST=*)
    local t=${s#TEST=}; local f=$O/pytest_$(basename ${t%%::*} .py).txt
    timeout -k 10 900 $PY -m pytest $t -m gpu -x -v --timeout 600 --timeout-method thread > $f 2>&1
    local rc=$?; tail -3 $f; return $rc ;;
  RUN=*)
    local spec=${s#RUN=}; local script=${spec%%,*}; local a=""
    [ "$spec" != "$script" ] && a=$(echo ${spec#*,} | tr ',' ' ')
    local f=$O/$(basename $script .py).jsonl
    timeout -k 10 900 $PY $script $a > $f 2> ${f%.jsonl}.err
    local rc=$?; tail -c 1500 $f; return $rc ;;
  smoke)
    timeout -k 10 300 $PY -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
    local rc=$?; tail -1 $O/smoke.txt; return $rc ;;
  bench)
    timeout -k 10 600 $PY bench.py > $O/bench.json 2> $O/bench.err
    local rc=$?; tail -c 600 $O/bench.json; echo; return $rc ;;
  jlprof)
    mkdir -p $O/jl
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/jl/prof -o run -- python3 $R/bench.py $JLARGS > $O/jl/prof_bench.json 2> $O/jl/prof.err) ;;
  jlpmc)
    mkdir -p $O/jl
    (cd /tmp && export TMPDIR=/tmp &&
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/jl/pmc_fetch -o run -- \
        python3 $R/bench.py $JLARGS > /dev/null 2> $O/jl/pmc_fetch.err &&
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/jl/pmc_write -o run -- \
        python3 $R/bench.py $JLARGS > /dev/null 2> $O/jl/pmc_write.err) ;;
  lompmc)
    mkdir -p $O/lom
    (cd /tmp && export TMPDIR=/tmp &&
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lom/prof -o run -- \
        python3 $R/bench.py $LOMARGS > $O/lom/prof_bench.json 2> $O/lom/prof.err &&
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/lom/pmc_fetch -o run -- \
        python3 $R/bench.py $LOMARGS > /dev/null 2> $O/lom/pmc_fetch.err &&
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/lom/pmc_write -o run -- \
        python3 $R/bench.py $LOMARGS > /dev/null 2> $O/lom/pmc_write.err)
    local rc=$?; tail -c 800 $O/lom/prof_bench.json; echo; return $rc ;;
  dist8|dist8full)
    local a="--elements 2000000 --steps 2 --warmup 1"
    [ $s = dist8full ] && a="--elements 10000000 --steps 20 --warmup 5"
    local t0=$(date +%s)
    timeout -k 10 900 $PY bench.py --gpus 8 --dist-backend gloo $a > $O/$s.json 2> $O/$s.err
    local rc=$?
    echo "{\"step\": \"$s\", \"rc\": $rc, \"wall_s\": $(( $(date +%s) - t0 )), \"lines\": $(wc -l < $O/$s.json)}" \
      > $O/$s.meta.json
    cat $O/$s.meta.json; holders | tee -a $O/$s.meta.json; tail -c 400 $O/$s.json; echo
    [ $rc -ne 0 ] && tail -c 2000 $O/$s.err
    return $rc ;;
  dist8run)
    local t0=$(date +%s)
    timeout -k 10 900 $PY -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 8 --dist-backend gloo --elements 2000000 --steps 2 --warmup 1 \
      > $O/$s.json 2> $O/$s.err
    local rc=$?
    echo "{\"step\": \"$s\", \"rc\": $rc, \"wall_s\": $(( $(date +%s) - t0 )), \"json_lines\": $(grep -c '^{' $O/$s.json)}" \
      > $O/$s.meta.json
    cat $O/$s.meta.json; holders | tee -a $O/$s.meta.json; tail -c 400 $O/$s.json; echo
    [ $rc -ne 0 ] && tail -c 2000 $O/$s.err
    return $rc ;;
  *)
    echo "unknown step $s"; return 2 ;;
  esac
}

for s in "$@"; do
  echo "== $s"
  run_step $s || { rc=$?; echo "STEP $s FAILED rc=$rc"; exit $rc; }
done
echo "pass $TAG done"
