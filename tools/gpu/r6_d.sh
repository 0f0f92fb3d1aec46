#!/bin/bash
# Round 6: headroom for batches in flight on one GPU (two and three handles, each its own 1M-topic
# batch stream, against one) on this round's kernels; then the default bench line under a
# rocprofv3 kernel trace + stats (profile evidence for this tree) and the 16k-topic line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/d
mkdir -p $O
timeout -k 10 400 python -u tools/concurrency.py --handles 2 --steps 40 > $O/conc2.json 2> $O/conc2.err || { tail -20 $O/conc2.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 -u $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/$O/trace.json 2> $R/$O/trace.err || { tail -20 $R/$O/trace.err; exit 1; }
cd $R
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
