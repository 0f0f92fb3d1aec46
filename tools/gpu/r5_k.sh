# Round 5: the sharded begin with one synchronisation (export from k_desc, packed by k_xpack):
# shard parity tests, then --sim-shards 2 / 4 / 8 at 10M
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_dist_engine.py tests/test_gpu_scale.py -m gpu -v --timeout 800 --timeout-method thread \
  -k "shard or dist or eight" > $O/pytest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in 8 4 2; do
  timeout -k 10 400 python -u bench.py --sim-shards $k --steps 5 --warmup 2 --no-cpu > $O/sim$k.json 2> $O/sim$k.err || exit 1
done
exit $rc
