#!/bin/bash
# Round 6: kernel trace of the 10M Messages line (where the image build's time goes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/z
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench_messages.py --steps 5 --warmup 2 --no-cpu > $O/msg_10m.json 2> $O/msg_10m.err || exit 1
