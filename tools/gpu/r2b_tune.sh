# Tuning: span-format step under engine option settings (tools/tune_spans.py), 10M then 1M.
set -o pipefail
D=gpurun_out/${1:-r2b_tune}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -20 $D/parity.log; exit 1; }
tail -2 $D/parity.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "${2:-9=1;9=8}" > $D/tune_10m.jsonl 2> $D/tune_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_10m.err; exit 1; }
cat $D/tune_10m.jsonl
timeout -k 10 200 python -u tools/tune_spans.py --subs 1000000 --reps 2 --configs "${2:-9=1;9=8}" > $D/tune_1m.jsonl 2> $D/tune_1m.err || { echo "tune1m rc=$?"; exit 1; }
cat $D/tune_1m.jsonl
