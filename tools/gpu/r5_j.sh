# Round 5: the sharded step with one synchronisation at each end of it: shard parity tests,
# --sim-shards 8 / 4 / 2 at 10M; then the default bench line, config 2 and the 16k-topic batch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_dist_engine.py tests/test_gpu_scale.py -m gpu -v --timeout 800 --timeout-method thread \
  -k "shard or dist or eight" > $O/pytest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in 8 4 2; do
  timeout -k 10 400 python -u bench.py --sim-shards $k --steps 5 --warmup 2 --no-cpu > $O/sim$k.json 2> $O/sim$k.err || exit 1
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python -u bench.py --subs 1000000 --steps 20 --warmup 5 > $O/bench_config2_1m.json 2> $O/bench_config2_1m.err || exit 1
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
exit $rc
