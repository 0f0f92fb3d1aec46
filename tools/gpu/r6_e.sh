#!/bin/bash
# Round 6: the concurrent readers/updates test with the merge-record flush moved ahead of the sync
# plan; headroom for two batches in flight on one GPU; config 5 at 100M retained with the runs
# output and its work-counter roofline (oracle side from profiles/r05/msg100m_oracle.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/e
mkdir -p $O
MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp.out 2> $O/cpp.err || { echo "cpp rc=$?"; grep -v "mq slow" $O/cpp.err | tail -30; }
timeout -k 10 400 python -u tools/concurrency.py --handles 2 --steps 40 > $O/conc2.json 2> $O/conc2.err || { tail -20 $O/conc2.err; exit 1; }
timeout -k 10 700 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --oracle-file profiles/r05/msg100m_oracle.json > $O/msg_100m.json 2> $O/msg_100m.err || { tail -20 $O/msg_100m.err; exit 1; }
