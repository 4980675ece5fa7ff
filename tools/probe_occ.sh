R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/probe1
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/exp_probe.py --ct 1024,4096,8192,16384,24576,32768,41667,49152,65536 --reps 2 > $O/occ.jsonl 2> $O/occ.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/agg -o run -- python3 $R/tools/agg_scaling.py --sizes 1250000 --reps 2 > $O/agg.json 2> $O/agg.err
rc=$?; echo rc=$rc; cat $O/occ.jsonl $O/agg.json; exit $rc
