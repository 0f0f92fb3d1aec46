# Round 5: sharded validation (k_set with rank keys, the u32 export pack) —
# the sharded tests, then 8 / 4 / 2 simulated shards at 10M
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/xpack32
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_dist_engine.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_shard.log 2>&1 || exit 1
for k in 8 4 2; do
  timeout -k 10 400 python -u bench.py --sim-shards $k --steps 5 --warmup 2 --no-cpu > $O/sim$k.json 2> $O/sim$k.err || exit 1
done
