# round 4: is the one-lane launch's ~3 ms per round in the H-load code?  r4a (before the launch-bytes
# changes), new (shipped), v2 = shipped with the round-3 whole-row H load in the kernel (build/ab/v2.so), v3 =
# v2 with both nude digits stored (build/ab/v3.so); v2 / v3 run with FBM_COMPACT_H=0 (whole rows written).
# One-lane decryption-factor launches only, interleaved, one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4tr3}
mkdir -p $O
NEW=$GRAFT_REPO_ROOT/fedbiomed_amd/_lib/libfbm_secagg.so
for rep in 1 2; do
  for v in r4a new v2; do
    case $v in r4a) L=build/ab/r4a.so; E="";; new) L=fedbiomed_amd/_lib/libfbm_secagg.so; E="";; *) L=build/ab/$v.so; E="FBM_COMPACT_H=0";; esac
    env FBM_LIB_PATH=$GRAFT_REPO_ROOT/$L $E timeout -k 10 200 python -u tools/exp_probe.py --ct 65536,131072 --engines single --reps 3 > $O/probe_$v.$rep.jsonl 2>&1 || { echo "PROBE FAILED $v"; tail -3 $O/probe_$v.$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep ct $O/probe_$v.$rep.jsonl
  done
done
