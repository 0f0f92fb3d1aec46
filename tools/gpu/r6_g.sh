#!/bin/bash
# Round 6: the C++ mirror alone with MQ_SLOW_MS milestones (a prepare phase without HIP calls under
# the host-image lock), then the whole GPU suite with per-test durations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/g2
mkdir -p $O
MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp.out 2> $O/cpp.err || { echo "cpp rc=$?"; grep -v "mq slow" $O/cpp.err | tail -30; }
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
