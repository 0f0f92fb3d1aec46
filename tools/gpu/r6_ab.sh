#!/bin/bash
# Round 6: work items of 64 particles / entries (lib_alt, MQ_MSG_CHUNK=64) against 256, 10M and
# 100M retained, A B A B; B's parity over every filter at 100M
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/ab
mkdir -p $O
ALT=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_alt
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/a10.json 2> $O/a10.err || exit 1
MQ_LIB_DIR=$ALT timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/b10.json 2> $O/b10.err || exit 1
timeout -k 10 400 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --no-cpu > $O/a100.json 2> $O/a100.err || exit 1
MQ_LIB_DIR=$ALT timeout -k 10 600 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --oracle-file profiles/r05/msg100m_oracle.json > $O/b100.json 2> $O/b100.err || exit 1
