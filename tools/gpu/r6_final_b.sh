#!/bin/bash
# Round 6 closing, part B: rocprofv3 kernel trace + stats of a short default run; the default bench
# line (CPU baseline, parity sample, end-to-end); the 16k-topic line with its host legs; config 2;
# 8 simulated shards
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/final
mkdir -p $O
# a line a minute under gpurun_out while the long steps build their 10M-subscription indexes in silence
( while true; do date >> $O/heartbeat.log; sleep 60; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $O/trace.json 2> $O/trace.err || exit 1
cd $R
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
timeout -k 10 300 python -u bench.py --subs 1000000 --steps 20 --warmup 5 > $O/bench_config2_1m.json 2> $O/bench_config2_1m.err || exit 1
timeout -k 10 400 python -u bench.py --sim-shards 8 --steps 20 --warmup 3 --no-cpu > $O/sim8.json 2> $O/sim8.err || exit 1
