#!/bin/bash
# Round 6: k_msgq's wide-count and place passes at 6 waves per SIMD (lib_alt, MQ_MSGQ_WAVES_OTHER=6)
# against the default register allocation (5), 10M and 100M retained, A B A
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/r
mkdir -p $O
ALT=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_alt
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/a1.json 2> $O/a1.err || exit 1
MQ_LIB_DIR=$ALT timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/b1.json 2> $O/b1.err || exit 1
timeout -k 10 300 python -u bench_messages.py --steps 20 --warmup 3 --no-cpu > $O/a2.json 2> $O/a2.err || exit 1
MQ_LIB_DIR=$ALT timeout -k 10 600 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --oracle-file profiles/r05/msg100m_oracle.json > $O/b100.json 2> $O/b100.err || exit 1
timeout -k 10 600 python3 -u bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 10 --warmup 3 --no-cpu > $O/a100.json 2> $O/a100.err || exit 1
