# Round 3: the GPU suite on the current tree (one-sync batches, sharded dedup, 8-shard config-3
# test), then one-sync vs host-synchronised batches at 10M.
set -o pipefail
D=gpurun_out/${1:-r3c}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|error" $D/pytest_gpu.log | head -20; tail -30 $D/pytest_gpu.log; exit 1; }
tail -3 $D/pytest_gpu.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "16=1;16=0" > $D/tune_sync_10m.jsonl 2> $D/tune_sync_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_sync_10m.err; exit 1; }
cat $D/tune_sync_10m.jsonl
