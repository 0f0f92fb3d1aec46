# Config 5 at full size, CPU side: the oracle's sample digests, counters and CPU baseline for
# 100M retained + 1k $SYS, 100k filters (bench_messages.py --oracle-only; no GPU use).
set -o pipefail
D=gpurun_out/${1:-r2c_msg100o}
mkdir -p $D
timeout -k 10 1080 python -u bench_messages.py --retained 100000000 --oracle-only $D/msg100m_oracle.json 2> $D/oracle.err || { echo "oracle rc=$?"; tail -5 $D/oracle.err; exit 1; }
grep -v working $D/oracle.err | tail -5
