# Round 2: the large configurations — config 4 IoT fan-in (50M subscriptions) and config 5 at its
# full size (100M retained + 1k $SYS, 100k filters) — and the default bench line.
set -o pipefail
D=gpurun_out/${1:-r2b_big}
mkdir -p $D
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_10m.json 2> $D/bench_10m.err || { echo "bench rc=$?"; tail -5 $D/bench_10m.err; exit 1; }
python tools/show.py $D/bench_10m.json
timeout -k 10 500 python -u bench.py --mix iot --subs 50000000 --no-cpu > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -5 $D/bench_iot_50m.err; exit 1; }
python tools/show.py $D/bench_iot_50m.json
timeout -k 10 600 python -u bench_messages.py --retained 100000000 --no-cpu > $D/msg_100m.json 2> $D/msg_100m.err || { echo "msg rc=$?"; tail -5 $D/msg_100m.err; exit 1; }
cat $D/msg_100m.json
