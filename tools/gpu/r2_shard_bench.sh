# Sharded mode on one GPU: 2 and 4 simulated shards at 10M subscriptions (per-shard work and the
# exchange volume), and the replicated default line for comparison.
set -o pipefail
D=gpurun_out/${1:-r2_shard}
mkdir -p $D
for G in 2 4; do
  timeout -k 10 600 python bench.py --sim-shards $G --steps 5 --warmup 2 > $D/bench_sim$G.json 2> $D/bench_sim$G.err || exit 1
  cat $D/bench_sim$G.json
done
