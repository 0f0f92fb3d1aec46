#!/bin/bash
# Round 6 closing, part A: the whole GPU suite with per-test durations, smoke(), the C++ mirror
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/final
mkdir -p $O
# a line a minute under gpurun_out while the long steps build their 10M-subscription indexes in silence
( while true; do date >> $O/heartbeat.log; sleep 60; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp.out 2> $O/cpp.err || { echo "cpp rc=$?"; exit 1; }
