# round 3, short path: the engine sweep (refit of engine_model_ms) and the one-box strong-scaling
# prediction (tools/predict_scaling.sh); each GPU step under its own time limit
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sweep
mkdir -p $O
timeout -k 10 400 python -u tools/exp_probe.py --ct 10752,21504,32256,43008,64512,86016,107520,131072,196608,262144 --engines triple,quad,single --reps 2 > $O/sweep.jsonl 2>&1 || { echo "SWEEP FAILED"; tail -5 $O/sweep.jsonl; exit 1; }
cat $O/sweep.jsonl | grep ct
timeout -k 10 900 bash tools/predict_scaling.sh predict_r3g > $O/predict.log 2>&1 || { echo "PREDICT FAILED"; tail -5 $O/predict.log; exit 1; }
cat $O/predict.log
