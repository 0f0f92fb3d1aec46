#!/bin/bash
# Round 6: entry-range work items (exported key-index levels): parity on every Messages test, then
# the export threshold A/B at 10M retained (512 default / 128 / 256 / 64)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "messages" tests/test_gpu_scale.py::test_messages_10m_retained_100k_filters -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { tail -30 $O/pytest_msg.log; exit 1; }
for x in 1 128 256 64; do
  timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu --export $x > $O/msg_10m_x$x.json 2> $O/msg_10m_x$x.err || { tail -20 $O/msg_10m_x$x.err; exit 1; }
done
