# Round 3: device-side batch order (MQ_OPT_TOPIC_ORDER): parity, then the 10M step with and
# without it, and against a host byte-sorted batch.
set -o pipefail
D=gpurun_out/${1:-r3g}
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "topic_order or one_sync or spans" > $D/pytest_order.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest_order.log; exit 1; }
tail -3 $D/pytest_order.log
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "17=1;17=0" > $D/order_10m.jsonl 2> $D/order_10m.err || { echo "tune rc=$?"; tail -5 $D/order_10m.err; exit 1; }
cut -c1-520 $D/order_10m.jsonl
