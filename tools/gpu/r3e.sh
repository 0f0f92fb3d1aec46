# Round 3: merge set pass register budget with 4 partner links per batch (was 8), Messages at 10M
# retained (level-synchronous fan-out), counters available on the box.
set -o pipefail
D=gpurun_out/${1:-r3e}
mkdir -p $D
timeout -s KILL 60 rocprofv3 -L > $D/counters_avail.txt 2>&1 || echo "list rc=$?"
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "7=8;7=6;7=1" > $D/tune_merge_wpe.jsonl 2> $D/tune_merge_wpe.err || { echo "tune rc=$?"; tail -5 $D/tune_merge_wpe.err; exit 1; }
cut -c1-330 $D/tune_merge_wpe.jsonl
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread -k "messages or msg or Messages" > $D/pytest_msg.log 2>&1 || { echo "pytest msg rc=$?"; tail -30 $D/pytest_msg.log; exit 1; }
tail -2 $D/pytest_msg.log
timeout -k 10 400 python -u bench_messages.py --retained 10000000 > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -5 $D/msg_10m.err; exit 1; }
cut -c1-700 $D/msg_10m.json
