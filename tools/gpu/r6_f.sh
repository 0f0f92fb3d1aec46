#!/bin/bash
# Round 6: HBM traffic of the Messages step with runs at the boundary, 100M retained x 100k filters
# (config 5): FETCH_SIZE and WRITE_SIZE of the k_msgq passes, one counter per rocprofv3 run
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/f
mkdir -p $O
MARGS="--retained 100000000 --sys 1000 --filters 100000 --steps 2 --warmup 1 --no-cpu"
timeout -s KILL 550 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $O/mfetch -o run -- python3 $R/bench_messages.py $MARGS > $O/mfetch.json 2> $O/mfetch.err || exit 1
timeout -s KILL 550 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $O/mwrite -o run -- python3 $R/bench_messages.py $MARGS > $O/mwrite.json 2> $O/mwrite.err || exit 1
