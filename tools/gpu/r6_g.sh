#!/bin/bash
# Round 6: the whole GPU suite on this tree (lock split, runs, deep-tail refcount, IoT half load,
# 16k-topic 8-shard check) and smoke(); the C++ mirror alone with MQ_SLOW_MS milestones first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/g
mkdir -p $O
MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp.out 2> $O/cpp.err || { echo "cpp rc=$?"; grep -v "mq slow" $O/cpp.err | tail -30; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
