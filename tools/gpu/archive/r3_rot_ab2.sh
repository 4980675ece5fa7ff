# round 3: the triple square microbench and the real engines' launch times on ONE box
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 tools/microbench/tri_variants 200 > gpurun_out/tv3.jsonl 2>&1 || { echo "TV FAILED"; exit 1; }
grep -E '"(base|base_rot2|madsonly)"' gpurun_out/tv3.jsonl
for v in vcc rot; do
  FBM_LIB_PATH=$GRAFT_REPO_ROOT/build/ab/$v.so timeout -k 10 200 python -u tools/exp_probe.py --ct 21504,43008,64512 --engines triple --reps 3 > gpurun_out/rot_probe2_$v.jsonl 2>&1 || { echo "PROBE FAILED $v"; exit 1; }
  echo "== $v"; grep ct gpurun_out/rot_probe2_$v.jsonl
done
timeout -k 10 200 tools/microbench/oprate 2000 > gpurun_out/oprate3.jsonl 2>&1 && grep -E 'v_mad_u64_u32"|srot' gpurun_out/oprate3.jsonl
