# Round 2: k_merge<spans> with the pair header folded into GDesc and slot meta in PairSlot —
# GPU test suite, then the occupancy variants at 10M and 1M subscriptions.
set -o pipefail
D=gpurun_out/r2_tune1
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a $D/pytest_gpu.log
tail -3 $D/pytest_gpu.log
timeout -k 10 400 python tools/tune_spans.py --subs 10000000 --configs "7=1;7=6;7=8" > $D/tune_10m.jsonl 2> $D/tune_10m.err || exit 1
cat $D/tune_10m.jsonl
timeout -k 10 300 python tools/tune_spans.py --subs 1000000 --configs "7=1;7=6;7=8" > $D/tune_1m.jsonl 2> $D/tune_1m.err || exit 1
cat $D/tune_1m.jsonl
