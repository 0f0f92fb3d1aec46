# GPU parity suite, then the Messages bench at 10M retained (config 5 scaled); FULL=1 adds 100M.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/msgtest
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 400 python bench_messages.py --steps 5 --warmup 2 > $D/bench_messages_10m.json 2> $D/bench_messages_10m.err || exit 1
if [ -n "$FULL" ]; then
timeout -k 10 700 python bench_messages.py --retained 100000000 --steps 5 --warmup 1 --no-cpu > $D/bench_messages_100m.json 2> $D/bench_messages_100m.err || exit 1
fi
