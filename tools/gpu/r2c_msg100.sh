# Config 5 at full size on the GPU (100M retained + 1k $SYS, 100k filters), parity sample,
# counters and CPU baseline from the committed oracle-side file of the same workload.
set -o pipefail
D=gpurun_out/${1:-r2c_msg100}
mkdir -p $D
timeout -k 10 700 python -u bench_messages.py --retained 100000000 --oracle-file profiles/r02/msg100m_oracle.json > $D/msg_100m.json 2> $D/msg_100m.err || { echo "msg rc=$?"; tail -5 $D/msg_100m.err; exit 1; }
cut -c1-2500 $D/msg_100m.json
