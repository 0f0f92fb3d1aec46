# Round 5: the sharded begin (one synchronisation, the export from k_desc): shard parity tests, then
# --sim-shards 8 at 10M against the classic begin (MQ_OPT_ONE_SYNC 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_dist_engine.py tests/test_gpu_scale.py -m gpu -v --timeout 800 --timeout-method thread \
  -k "shard or dist or eight" > $O/pytest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 5 --warmup 2 --no-cpu > $O/sim8.json 2> $O/sim8.err || exit 1
MQ_ENGINE_OPTIONS=16=0 timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 5 --warmup 2 --no-cpu > $O/sim8_classic.json 2> $O/sim8_classic.err || exit 1
MQ_LIB_DIR=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_dev timeout -k 10 300 python -u tools/ab_options.py --check 4096 --variants 24=0 24=1 --rounds 3 > $O/ab_root.json 2> $O/ab_root.err || exit 1
exit $rc
