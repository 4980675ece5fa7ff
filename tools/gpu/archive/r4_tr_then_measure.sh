# the traffic A/B (tools/gpu/r4_traffic_ab.sh) and, if it passes, the measurement pass of the same library
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r4_traffic_ab.sh ${1:-r4tr} && SKIP_PYTEST=1 bash tools/gpu/r4_measure.sh ${2:-r4m}
