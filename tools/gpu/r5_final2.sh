# Round 5 final lines on the final tree: the default bench line (CPU baseline, parity sample,
# end-to-end), the 16k-topic batch, config 2, the simulated shards, and the rocprofv3 kernel
# trace + stats of a short default run
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/final2
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $O/trace.json 2> $O/trace.err || exit 1
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_dist_engine.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_shard.log 2>&1 || exit 1
timeout -k 10 120 ./mqtt-server_amd/build/test_topics_index > $O/cpp.out 2> $O/cpp.err; echo "cpp rc=$?" > $O/cpp_rc.txt
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
timeout -k 10 300 python -u bench.py --subs 1000000 --steps 20 --warmup 5 > $O/bench_config2_1m.json 2> $O/bench_config2_1m.err || exit 1
for k in 8 4 2; do
  timeout -k 10 400 python -u bench.py --sim-shards $k --steps 5 --warmup 2 --no-cpu > $O/sim$k.json 2> $O/sim$k.err || exit 1
done
