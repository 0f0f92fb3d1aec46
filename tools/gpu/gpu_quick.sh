# Quick GPU iteration: parity tests, then 1M and 10M benches (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/q/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --subs 1000000 --steps 5 --warmup 2 --no-cpu > gpurun_out/q/bench_1m.json 2> gpurun_out/q/bench_1m.err || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/q/bench_10m.json 2> gpurun_out/q/bench_10m.err || exit 1
MQ_MERGE_STATS=1 timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/q/stats_10m.json 2> gpurun_out/q/stats_10m.err || exit 1
