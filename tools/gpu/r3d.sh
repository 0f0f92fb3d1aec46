# Round 3: the distributed / sharded tests first (the last run stalled in the two-rank sharded
# test), then the whole GPU suite, then one-sync vs host-synchronised batches at 10M.
set -o pipefail
D=gpurun_out/${1:-r3d}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_dist_engine.py tests/test_gpu_shard.py -x -v --timeout 170 --timeout-method thread > $D/pytest_shard.log 2>&1 || { echo "pytest shard rc=$?"; tail -60 $D/pytest_shard.log; exit 1; }
tail -3 $D/pytest_shard.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread --deselect tests/test_dist_engine.py --deselect tests/test_gpu_shard.py > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $D/pytest_gpu.log; exit 1; }
tail -3 $D/pytest_gpu.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "16=1;16=0" > $D/tune_sync_10m.jsonl 2> $D/tune_sync_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_sync_10m.err; exit 1; }
cat $D/tune_sync_10m.jsonl
