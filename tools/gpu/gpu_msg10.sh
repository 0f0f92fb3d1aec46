# Messages bench at 10M retained (config 5 scaled), no CPU baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/msg10
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k messages -x -q --timeout 120 --timeout-method thread > $D/pytest_msg.log 2>&1 || exit 1
timeout -k 10 600 python bench_messages.py --retained 10000000 --filters 100000 --no-cpu > $D/msg_10m.json 2> $D/msg_10m.err || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu > $D/bench_10m_overlap.json 2> $D/bench_10m_overlap.err || exit 1
timeout -k 10 300 python bench.py --subs 1000000 --steps 10 --warmup 2 --no-cpu > $D/bench_1m.json 2> $D/bench_1m.err || exit 1
