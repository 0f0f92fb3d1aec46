# Round 3 (session 2): Messages with wide fan-outs exported to work items (MQ_OPT_MSG_EXPORT 19):
# the Messages parity tests, then 10M retained with and without the export (+ work counters).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3q}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "messages" -x -v --timeout 170 --timeout-method thread > $D/pytest_msg.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_msg.log; exit 1; }
tail -3 $D/pytest_msg.log
timeout -k 10 400 python -u tools/tune_msg.py --retained 10000000 --configs "19=1;19=0" --repeat 2 --work > $D/msgexp_10m.jsonl 2> $D/msgexp_10m.err || { echo "tune rc=$?"; tail -5 $D/msgexp_10m.err; exit 1; }
cat $D/msgexp_10m.jsonl
