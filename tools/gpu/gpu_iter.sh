# Iteration: parity tests, 1M and 10M benches (no CPU baseline), isolated-kernel 10M run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/it
D=gpurun_out/it
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --subs 1000000 --steps 5 --warmup 2 --no-cpu > $D/bench_1m.json 2> $D/bench_1m.err || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu > $D/bench_10m.json 2> $D/bench_10m.err || exit 1
MQ_SERIAL=1 timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu > $D/serial_10m.json 2> $D/serial_10m.err || exit 1
