# Round 3: the batching stage under 64 submitters (tools/latency.cpp) and the sharded step
# simulated on one GPU with 2, 4 and 8 shards at 10M subscriptions.
set -o pipefail
D=gpurun_out/${1:-r3h}
mkdir -p $D
timeout -k 10 300 mqtt-server_amd/build/latency 10000000 3 > $D/latency_10m.jsonl 2> $D/latency_10m.err || { echo "latency rc=$?"; tail -5 $D/latency_10m.err; exit 1; }
cat $D/latency_10m.jsonl
for S in 2 4 8; do
  timeout -k 10 420 python -u bench.py --sim-shards $S --steps 5 --warmup 2 --no-cpu > $D/bench_sim${S}_10m.json 2> $D/bench_sim${S}_10m.err || { echo "sim$S rc=$?"; tail -5 $D/bench_sim${S}_10m.err; exit 1; }
  cut -c1-1500 $D/bench_sim${S}_10m.json
done
