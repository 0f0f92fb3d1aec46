#!/bin/bash
# Round 6 closing, Messages: rocprofv3 kernel trace + stats of the 100M-retained line on the final
# kernels, then its HBM traffic (FETCH_SIZE, WRITE_SIZE, separate passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/x
mkdir -p $O
( while true; do date >> $O/heartbeat.log; sleep 60; done ) &
HB=$!
trap "kill $HB" EXIT
MARGS="--retained 100000000 --sys 1000 --filters 100000"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench_messages.py $MARGS --steps 10 --warmup 3 --no-cpu > $O/msg_100m_trace.json 2> $O/msg_100m_trace.err || exit 1
timeout -s KILL 550 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $O/mfetch -o run -- python3 $R/bench_messages.py $MARGS --steps 2 --warmup 1 --no-cpu > $O/mfetch.json 2> $O/mfetch.err || exit 1
timeout -s KILL 550 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $O/mwrite -o run -- python3 $R/bench_messages.py $MARGS --steps 2 --warmup 1 --no-cpu > $O/mwrite.json 2> $O/mwrite.err || exit 1
