# Parity suite, then a 1M bench line with the end-to-end (host-buffer) sample.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/e2e2
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --subs 1000000 --steps 5 --warmup 1 --cpu-seconds 3 > $D/bench_1m.json 2> $D/bench_1m.err || exit 1
timeout -k 10 500 python bench.py --steps 5 --warmup 2 --no-cpu > $D/bench_10m.json 2> $D/bench_10m.err || exit 1
