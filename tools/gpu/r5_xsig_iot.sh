# Round 5: the dedup insert inside k_xsig (sharded tests, 8 simulated shards), then config 4
# (50M IoT filters: the thread-per-topic walk) on the final kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/xsig_iot
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_dist_engine.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_shard.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 5 --warmup 2 --no-cpu > $O/sim8.json 2> $O/sim8.err || exit 1
timeout -k 10 800 python -u bench.py --mix iot --subs 50000000 --steps 10 --warmup 3 --no-cpu > $O/bench_iot_50m.json 2> $O/bench_iot_50m.err || exit 1
