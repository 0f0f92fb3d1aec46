# GPU session script: parity tests, 1M bench, kernel-trace profile, 10M bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --subs 1000000 --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/bench_1m.json 2> gpurun_out/bench_1m.err || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_1m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --subs 1000000 --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_1m.log 2>&1 ) || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-seconds 10 > gpurun_out/bench_10m.json 2> gpurun_out/bench_10m.err || exit 1
