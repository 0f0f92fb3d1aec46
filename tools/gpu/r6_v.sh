#!/bin/bash
# Round 6: the Messages count pass at 6 waves per SIMD (lib_alt, MQ_MSGQ_WAVES_RUNS=6: 80 VGPRs,
# 28 spilled) against 5 (96 VGPRs), 10M retained A B A B, then 100M B A
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/v
mkdir -p $O
ALT=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_alt
for k in 1 2; do
  timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/a$k.json 2> $O/a$k.err || exit 1
  MQ_LIB_DIR=$ALT timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/b$k.json 2> $O/b$k.err || exit 1
done
MQ_LIB_DIR=$ALT timeout -k 10 600 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --no-cpu > $O/b100.json 2> $O/b100.err || exit 1
timeout -k 10 600 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --no-cpu > $O/a100.json 2> $O/a100.err || exit 1
