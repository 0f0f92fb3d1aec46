#!/bin/bash
# Round 6: the C++ mirror's concurrent test three times (FifoMutex waiters spin before sleeping);
# HBM traffic of the Messages step at 100M retained with the key index (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/m
mkdir -p $O
for k in 1 2 3; do
  MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp$k.out 2> $O/cpp$k.err || { echo "cpp rc=$?"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
MARGS="--retained 100000000 --sys 1000 --filters 100000 --steps 2 --warmup 1 --no-cpu"
timeout -s KILL 550 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $R/$O/mfetch -o run -- python3 $R/bench_messages.py $MARGS > $R/$O/mfetch.json 2> $R/$O/mfetch.err || exit 1
timeout -s KILL 550 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $R/$O/mwrite -o run -- python3 $R/bench_messages.py $MARGS > $R/$O/mwrite.json 2> $R/$O/mwrite.err || exit 1
