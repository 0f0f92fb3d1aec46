#!/bin/bash
# Round 6: entry items exported above 128 candidate entries (the default now): Messages parity,
# 10M (default, and without the key index), 100M retained with every filter digest-checked, and
# the 100M step's HBM traffic (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "messages" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { tail -30 $O/pytest_msg.log; exit 1; }
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 > $O/msg_10m.json 2> $O/msg_10m.err || { tail -20 $O/msg_10m.err; exit 1; }
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu --no-key-index > $O/msg_10m_nokx.json 2> $O/msg_10m_nokx.err || { tail -20 $O/msg_10m_nokx.err; exit 1; }
timeout -k 10 700 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --oracle-file profiles/r05/msg100m_oracle.json > $O/msg_100m.json 2> $O/msg_100m.err || { tail -20 $O/msg_100m.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
MARGS="--retained 100000000 --sys 1000 --filters 100000 --steps 2 --warmup 1 --no-cpu"
timeout -s KILL 550 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $R/$O/mfetch -o run -- python3 $R/bench_messages.py $MARGS > $R/$O/mfetch.json 2> $R/$O/mfetch.err || exit 1
timeout -s KILL 550 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $R/$O/mwrite -o run -- python3 $R/bench_messages.py $MARGS > $R/$O/mwrite.json 2> $R/$O/mwrite.err || exit 1
