# GPU suite (incl. the C++ host mirror tests), update-path bench, batch latency sweep at 10M
set -o pipefail
D=gpurun_out/${1:-r2_lat}
mkdir -p $D
bash tools/gpu/r2_suite.sh ${1:-r2_lat} || exit 1
timeout -k 10 500 python -u tools/bench_update.py --subs 10000000 --retained 10000000 > $D/update.json 2> $D/update.err || { echo "update rc=$?"; tail -5 $D/update.err; exit 1; }
cat $D/update.json
timeout -k 10 400 ./mqtt-server_amd/build/latency 10000000 3 > $D/latency.jsonl 2> $D/latency.err || { echo "latency rc=$?"; tail -5 $D/latency.err; exit 1; }
cat $D/latency.jsonl
