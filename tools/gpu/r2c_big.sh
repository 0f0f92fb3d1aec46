# Config 5 at full size (100M retained + 1k $SYS): host/device image checks and one Messages
# batch both ways (tools/diag_msg.py), then the config-5 bench line; config 4 (50M IoT) bench.
set -o pipefail
D=gpurun_out/${1:-r2c_big}
mkdir -p $D
timeout -k 10 500 python -u tools/diag_msg.py 100000000 > $D/diag_msg.log 2>&1; rc=$?; echo "diag rc=$rc"; cut -c1-300 $D/diag_msg.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u bench_messages.py --retained 100000000 > $D/msg_100m.json 2> $D/msg_100m.err || { echo "msg rc=$?"; tail -5 $D/msg_100m.err; exit 1; }
cut -c1-1500 $D/msg_100m.json
