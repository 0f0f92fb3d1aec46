#!/bin/bash
# Round 6: (1) the C++ mirror's concurrent test twice (slowest update once the readers are warm);
# (2) the Messages key index A/B at 10M retained (on, off, on); (3) 100M retained with the key index,
# every filter digest-checked against the oracle's file; (4) its HBM traffic (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/k
mkdir -p $O
for k in 1 2; do
  MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp$k.out 2> $O/cpp$k.err || { echo "cpp rc=$?"; exit 1; }
done
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/msg_10m_kx.json 2> $O/msg_10m_kx.err || { tail -20 $O/msg_10m_kx.err; exit 1; }
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu --no-key-index > $O/msg_10m_nokx.json 2> $O/msg_10m_nokx.err || { tail -20 $O/msg_10m_nokx.err; exit 1; }
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/msg_10m_kx2.json 2> $O/msg_10m_kx2.err || { tail -20 $O/msg_10m_kx2.err; exit 1; }
timeout -k 10 700 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --oracle-file profiles/r05/msg100m_oracle.json > $O/msg_100m.json 2> $O/msg_100m.err || { tail -20 $O/msg_100m.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
MARGS="--retained 100000000 --sys 1000 --filters 100000 --steps 2 --warmup 1 --no-cpu"
timeout -s KILL 550 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $R/$O/mfetch -o run -- python3 $R/bench_messages.py $MARGS > $R/$O/mfetch.json 2> $R/$O/mfetch.err || exit 1
timeout -s KILL 550 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_msgq" --output-format csv -d $R/$O/mwrite -o run -- python3 $R/bench_messages.py $MARGS > $R/$O/mwrite.json 2> $R/$O/mwrite.err || exit 1
