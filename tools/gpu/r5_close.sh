# Round 5: the tree as committed last (the fold's fill experiment bits built in, off by default):
# set-pass and sharded parity, smoke(), the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/close
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -x -v --timeout 200 --timeout-method thread -k "set_pass or spans or merging or pair_hits or partner_map or long_lists or workload_digest or shard or config3 or deep or golden or kat" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
