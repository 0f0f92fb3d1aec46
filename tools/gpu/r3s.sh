# Round 3 (session 2): Messages wide items with recorded runs (no second walk): Messages parity
# tests, then the export thresholds at 10M retained.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3s}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "messages" -x -v --timeout 170 --timeout-method thread > $D/pytest_msg.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_msg.log; exit 1; }
tail -3 $D/pytest_msg.log
timeout -k 10 400 python -u tools/tune_msg.py --retained 10000000 --configs "19=2048;19=1024;19=512;19=256;19=0" --repeat 2 --work > $D/msgthr_10m.jsonl 2> $D/msgthr_10m.err || { echo "tune rc=$?"; tail -5 $D/msgthr_10m.err; exit 1; }
cut -c1-700 $D/msgthr_10m.jsonl
