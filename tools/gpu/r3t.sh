# Round 3 (session 2): one-sync batches with one k_reset and one k_readback (no fill / copy
# commands), Messages wide items with recorded runs: smoke, the parity file, the 10M step, and
# the Messages export thresholds at 10M retained.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3t}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 170 --timeout-method thread > $D/pytest_parity.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_parity.log; exit 1; }
tail -3 $D/pytest_parity.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "17=1" > $D/step_10m.jsonl 2> $D/step_10m.err || { echo "tune rc=$?"; tail -5 $D/step_10m.err; exit 1; }
cut -c1-600 $D/step_10m.jsonl
timeout -k 10 400 python -u tools/tune_msg.py --retained 10000000 --configs "19=2048;19=512;19=0" --repeat 2 --work > $D/msgthr_10m.jsonl 2> $D/msgthr_10m.err || { echo "tune rc=$?"; tail -5 $D/msgthr_10m.err; exit 1; }
cut -c1-700 $D/msgthr_10m.jsonl
