# Round 5: the sharded k_set with the 192-word extra table (fold caps 240 / 480 visits), the sharded
# bench without events in its timed steps; A/B of MQ_OPT_SET_EXP bit 16 (the hash fold at most 2/3
# full) at 1M and 16k topics; the visits' pair slots loaded two rounds ahead; set-pass and sharded parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/fold2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -x -v --timeout 200 --timeout-method thread -k "set_pass or spans or merging or pair_hits or partner_map or long_lists or workload_digest or shard or config3 or deep" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 20 --warmup 3 --no-cpu > $O/sim8.json 2> $O/sim8.err || exit 1
timeout -k 10 300 python -u tools/ab_options.py --variants 18=0 18=65536 --rounds 3 --check 20000 > $O/ab_1m.json 2> $O/ab_1m.err || exit 1
timeout -k 10 300 python -u tools/ab_options.py --topics 16384 --steps 100 --variants 18=0 18=65536 --rounds 3 --check 16384 > $O/ab_16k.json 2> $O/ab_16k.err || exit 1
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || exit 1
