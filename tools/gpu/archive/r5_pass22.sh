# round 5, pass 22: the factor-ahead encrypt's kernels (rocprofv3 kernel trace) and the prepare tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r5ao}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_encrypt_factor.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_encf.txt 2>&1 || { echo "ENCF FAILED"; grep -E "FAILED|Error|assert" $O/pytest_encf.txt | head -30; exit 1; }
tail -1 $O/pytest_encf.txt
timeout -k 10 200 python -u tools/encf_probe.py > $O/encf_probe.jsonl 2>&1 || { echo "PROBE FAILED"; tail -20 $O/encf_probe.jsonl; exit 1; }
cat $O/encf_probe.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/encf_probe.py --elements 10000000 --reps 3 > $O/prof_probe.txt 2> $O/prof.err
