# round 3: the group engines with one copy of the unrolled cyclic-band square (the table path on the looped
# square: 87 / 106 KB kernels) vs three copies (build/ab/shortonly.so's group kernels: 108 / 133 KB) -- the
# full -m gpu suite on the shipped library first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gcode
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
lib() { case $1 in new) echo $GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so;; *) echo $GRAFT_REPO_ROOT/build/ab/$1.so;; esac; }
for rep in 1 2; do
  for v in shortonly new; do
    FBM_LIB_PATH=$(lib $v) timeout -k 10 200 python -u tools/exp_probe.py --ct 21504,41667,83334 --engines triple,quad --reps 2 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl
  done
done
