# Sharded k_merge without scratch: sharded GPU tests, then 2/4 simulated shards at 10M.
set -o pipefail
D=gpurun_out/${1:-r2_shard2}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_dist_engine.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
echo "pytest rc=$?"; tail -2 $D/pytest.log
for G in 2 4; do
  timeout -k 10 600 python bench.py --sim-shards $G --steps 5 --warmup 2 > $D/bench_sim$G.json 2> $D/bench_sim$G.err || exit 1
  cat $D/bench_sim$G.json
done
