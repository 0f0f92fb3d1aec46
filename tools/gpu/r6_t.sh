#!/bin/bash
# Round 6: the Messages count pass's per-filter clocks (total, p50, p99, max, heaviest 1 % / 0.1 %)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/t
mkdir -p $O
timeout -k 10 300 python -u bench_messages.py --steps 10 --warmup 3 --no-cpu > $O/msg_10m.json 2> $O/msg_10m.err || exit 1
timeout -k 10 600 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 5 --warmup 2 --no-cpu > $O/msg_100m.json 2> $O/msg_100m.err || exit 1
