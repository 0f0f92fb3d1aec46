# Round 5: kernel arguments read from the kernarg segment at their uses (k_walkf's fused desc,
# k_set, k_merge: no scalar-register spills to vector lanes), the deep-path tie-break compiled
# only into the kernels of indexes with deep filters — parity, the C++ mirror, then the default,
# 16k and 8-shard lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/kernarg2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 5 --warmup 2 --no-cpu > $O/sim8.json 2> $O/sim8.err || exit 1
exit $rc
