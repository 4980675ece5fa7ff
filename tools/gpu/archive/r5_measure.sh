# round 5 measurement pass (gpurun, from the repo root): LOM aggregate variants at config-5 shape, the
# MFMA i8 lane-map probe, config 5 (tools/bench_cfg5.py) with its kernel trace, HBM-traffic and SQ
# counter passes, and the JL 10M step's kernel trace + HBM-traffic passes.  Each GPU step has its own
# limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5b}
mkdir -p $O/cfg5 $O/jl
cd $R
timeout -k 10 60 ./tools/microbench/mfma_i8_map > $O/mfma_i8_map.txt 2>&1 || { echo "MFMA MAP FAILED"; cat $O/mfma_i8_map.txt; exit 1; }
cat $O/mfma_i8_map.txt
timeout -k 10 300 ./tools/microbench/agg_variants 100000000 16 7 > $O/agg_variants.jsonl 2>&1 || { echo "AGG VARIANTS FAILED"; tail -5 $O/agg_variants.jsonl; exit 1; }
tail -14 $O/agg_variants.jsonl
timeout -k 10 300 python -u tools/bench_cfg5.py > $O/cfg5_bench.json 2> $O/cfg5_bench.err || { echo "CFG5 FAILED"; tail -5 $O/cfg5_bench.err; exit 1; }
cat $O/cfg5_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg5/prof -o run -- python3 $R/tools/bench_cfg5.py --reps 1 > /dev/null 2> $O/cfg5/prof.err &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cfg5/pmc_fetch -o run -- python3 $R/tools/bench_cfg5.py --reps 1 > /dev/null 2> $O/cfg5/fetch.err &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cfg5/pmc_write -o run -- python3 $R/tools/bench_cfg5.py --reps 1 > /dev/null 2> $O/cfg5/write.err &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/cfg5/pmc_sq -o run -- python3 $R/tools/bench_cfg5.py --reps 1 > /dev/null 2> $O/cfg5/sq.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/jl/prof -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > $O/jl/prof_bench.json 2> $O/jl/prof.err &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/jl/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $O/jl/fetch.err &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/jl/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --serial --no-cpu-baseline --no-lom-extra --no-e2e --no-stages > /dev/null 2> $O/jl/write.err
rc=$?
echo "rc=$rc"
exit $rc
