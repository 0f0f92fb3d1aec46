# Round 2: update path (bulk build, churn + mq_sync), batch latency sweep, sharded mode simulated
# on one GPU (2 and 4 shards), config-1 (10k subscriptions). Each step under its own time limit.
set -o pipefail
D=gpurun_out/${1:-r2b_misc}
mkdir -p $D
timeout -k 10 420 python -u tools/bench_update.py --subs 10000000 --retained 10000000 > $D/update.json 2> $D/update.err || { echo "update rc=$?"; tail -5 $D/update.err; exit 1; }
cat $D/update.json
timeout -k 10 300 ./mqtt-server_amd/build/latency 10000000 3 > $D/latency.jsonl 2> $D/latency.err || { echo "latency rc=$?"; tail -5 $D/latency.err; exit 1; }
cat $D/latency.jsonl
for G in 2 4; do
  timeout -k 10 240 python -u bench.py --sim-shards $G --steps 5 --warmup 2 > $D/bench_sim$G.json 2> $D/bench_sim$G.err || { echo "sim$G rc=$?"; tail -5 $D/bench_sim$G.err; exit 1; }
  cat $D/bench_sim$G.json
done
timeout -k 10 200 python -u bench.py --subs 10000 --steps 10 --warmup 3 > $D/bench_config1.json 2> $D/bench_config1.err || { echo "config1 rc=$?"; exit 1; }
cat $D/bench_config1.json
