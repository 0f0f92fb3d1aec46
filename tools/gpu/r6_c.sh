#!/bin/bash
# Round 6: (1) the C++ mirror's concurrent readers/updates test with the sync's allocations made
# outside the host-image lock (MQ_SLOW_MS milestones); (2) Messages runs at the boundary — the
# runs parity tests and the 10M GPU test, then config 5 at 10M (oracle side in process) and at its
# full 100M retained (oracle side from profiles/r05/msg100m_oracle.json, same generator and seeds)
# under a rocprofv3 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/c
mkdir -p $O
MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp.out 2> $O/cpp.err || { echo "cpp rc=$?"; grep -v "mq slow" $O/cpp.err | tail -30; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "messages" tests/test_gpu_scale.py::test_messages_10m_retained_100k_filters -m gpu -x -v --timeout 500 --timeout-method thread > $O/pytest_msg.log 2>&1 || { tail -30 $O/pytest_msg.log; exit 1; }
timeout -k 10 400 python -u bench_messages.py --steps 10 --warmup 3 > $O/msg_10m.json 2> $O/msg_10m.err || { tail -20 $O/msg_10m.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 -u $R/bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 5 --warmup 2 --oracle-file $R/profiles/r05/msg100m_oracle.json > $R/$O/msg_100m.json 2> $R/$O/msg_100m.err || { tail -20 $R/$O/msg_100m.err; exit 1; }
