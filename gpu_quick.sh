# Quick GPU iteration: parity tests, then 1M and 10M benches with the k_emit wave profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/q/pytest_gpu.log 2>&1 || exit 1
MQ_EMIT_PROF=1 timeout -k 10 300 python bench.py --subs 1000000 --steps 2 --warmup 0 --no-cpu > gpurun_out/q/wprof_1m.json 2> gpurun_out/q/wprof_1m.err || exit 1
timeout -k 10 300 python bench.py --subs 1000000 --steps 5 --warmup 2 --no-cpu > gpurun_out/q/bench_1m.json 2> gpurun_out/q/bench_1m.err || exit 1
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/q/bench_10m.json 2> gpurun_out/q/bench_10m.err || exit 1
