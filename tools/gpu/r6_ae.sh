#!/bin/bash
# Round 6: the key index's try threshold 3 against 6 (default), 10M and 100M, A B A B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/ae
mkdir -p $O
for r in 6 3 6 3; do
  timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu --key-index-rounds $r > $O/m10.json 2> $O/m10.err || exit 1
  cp $O/m10.json $O/m10_r${r}_$(date +%s).json
done
for r in 6 3; do
  timeout -k 10 400 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --no-cpu --key-index-rounds $r > $O/m100_r$r.json 2> $O/m100_r$r.err || exit 1
done
