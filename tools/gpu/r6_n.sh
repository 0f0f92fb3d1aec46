#!/bin/bash
# Round 6: the key index's cost model (searches + hit rounds against the particles' probe rounds)
# and its try threshold (rounds of particle probes): parity on every Messages test, then 10M
# retained at thresholds 12 (default) / 24 / 48 / 6 and without the index, 100M at the default
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "messages" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { tail -30 $O/pytest_msg.log; exit 1; }
for r in 12 24 48 6; do
  timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu --key-index-rounds $r > $O/msg_10m_r$r.json 2> $O/msg_10m_r$r.err || { tail -20 $O/msg_10m_r$r.err; exit 1; }
done
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu --no-key-index > $O/msg_10m_nokx.json 2> $O/msg_10m_nokx.err || { tail -20 $O/msg_10m_nokx.err; exit 1; }
timeout -k 10 700 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --oracle-file profiles/r05/msg100m_oracle.json > $O/msg_100m.json 2> $O/msg_100m.err || { tail -20 $O/msg_100m.err; exit 1; }
