# Round 5 (final kernels): config 5 at its stated size — 100M retained topics (+1k $SYS) x 100k
# wildcard filters, parity against the --oracle-only side produced in its own call
# (profiles/r05/msg100m_oracle.json: fast-restatement digests of every filter, pinned to the
# oracle on 4,096), under a rocprofv3 kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/m100b
mkdir -p $O
timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u $R/bench_messages.py --retained 100000000 --sys 1000 --filters 100000 --steps 5 --warmup 2 --oracle-file $R/profiles/r05/msg100m_oracle.json > $O/msg_100m.json 2> $O/msg_100m.err || exit 1
