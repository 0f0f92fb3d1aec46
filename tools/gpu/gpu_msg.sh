# Parity suite, then the Messages bench (config 5 scaled).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/msg4
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench_messages.py --retained 1000000 --filters 100000 > $D/msg_1m.json 2> $D/msg_1m.err || exit 1
timeout -k 10 600 python bench_messages.py --retained 10000000 --filters 100000 > $D/msg_10m.json 2> $D/msg_10m.err || exit 1
