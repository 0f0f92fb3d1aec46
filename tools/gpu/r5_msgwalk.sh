# Round 5: k_msgq and k_walk with their DevIndex / image arguments read from the kernarg segment
# at their uses — the GPU suite's parity and Messages tests, then Messages at 10M retained, the
# default line, and config 4 (50M IoT filters, the thread-per-topic walk)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/msgwalk
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench_messages.py > $O/msg_10m.json 2> $O/msg_10m.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 700 python -u bench.py --mix iot --subs 50000000 --steps 10 --warmup 3 --no-cpu > $O/bench_iot_50m.json 2> $O/bench_iot_50m.err || exit 1
