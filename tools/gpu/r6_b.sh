#!/bin/bash
# Round 6: the handle lock split (updates never wait for a match's GPU work): the parity suite and
# the C++ mirror's concurrent readers/updates test (MQ_SLOW_MS milestones); then config 4 re-pinned
# — the IoT index at half edge-table load against the oracle, and the 50M IoT bench line with its
# oracle side on (20k-topic parity sample, roofline, CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/b
mkdir -p $O
MQ_SLOW_MS=2 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp.out 2> $O/cpp.err || { echo "cpp rc=$?"; tail -30 $O/cpp.err; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -k "iot" -m gpu -x -v --timeout 450 --timeout-method thread > $O/pytest_iot.log 2>&1 || { tail -30 $O/pytest_iot.log; exit 1; }
timeout -k 10 900 python -u bench.py --mix iot --subs 50000000 --steps 10 --warmup 3 > $O/bench_iot_50m.json 2> $O/bench_iot_50m.err || exit 1
