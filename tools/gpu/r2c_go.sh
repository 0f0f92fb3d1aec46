# Wave-leader dedup insert + representative list: parity (dedup on), span step dedup on/off at
# 10M and 1M; then config 5 at full size with the grid-stride image build (bench_messages.py,
# 100M retained + 1k $SYS, 100k filters).
set -o pipefail
D=gpurun_out/${1:-r2c_go}
mkdir -p $D
MQ_ENGINE_OPTIONS=12=1 bash tools/gpu/r2b_tune.sh ${1:-r2c_go} "12=1;12=0" || exit 1
timeout -k 10 600 python -u bench_messages.py --retained 100000000 > $D/msg_100m.json 2> $D/msg_100m.err || { echo "msg rc=$?"; tail -5 $D/msg_100m.err; exit 1; }
cut -c1-2000 $D/msg_100m.json
