#!/bin/bash
# Round 6 closing, Messages on the final tree: parity (every Messages test), the 10M line with the
# oracle side, the 100M line with every filter digest-checked
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/ad
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "messages" tests/test_gpu_scale.py::test_messages_10m_retained_100k_filters -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { tail -30 $O/pytest_msg.log; exit 1; }
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 > $O/msg_10m.json 2> $O/msg_10m.err || exit 1
timeout -k 10 700 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --oracle-file profiles/r05/msg100m_oracle.json > $O/msg_100m.json 2> $O/msg_100m.err || exit 1
