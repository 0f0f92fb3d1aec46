#!/bin/bash
# Round 6: the export threshold at 100M retained (default 512 particles / 128 hits; N sets both)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/aa
mkdir -p $O
for x in 1 256 64 1; do
  timeout -k 10 400 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --no-cpu --export $x > $O/msg_100m_x$x.json 2> $O/msg_100m_x$x.err || exit 1
  cp $O/msg_100m_x$x.json $O/msg_100m_x${x}_$(date +%s).json
done
