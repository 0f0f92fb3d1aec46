# Round 5: k_set's pair analysis two rounds at a time (first probes loaded together) — set-pass
# and sharded parity, then the default, 16k and 8-shard lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/pairs
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -x -v --timeout 200 --timeout-method thread -k "set_pass or spans or merging or pair_hits or partner_map or long_lists or workload_digest or shard or config3 or deep" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 5 --warmup 2 --no-cpu > $O/sim8.json 2> $O/sim8.err || exit 1
