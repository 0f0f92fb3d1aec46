#!/bin/bash
# Round 6: the export threshold with the key index (hits above it go to work items), 10M retained
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/o
mkdir -p $O
for x in 1 128 2048 8192 1; do
  timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu --export $x > $O/msg_10m_x$x.json 2> $O/msg_10m_x$x.err || { tail -20 $O/msg_10m_x$x.err; exit 1; }
done
