# Round 5: the sharded step after the walk's instruction work — kernel timeline of 8 simulated
# shards at 10M (gaps: host work per shard), the sim lines at 8 / 4 / 2 shards, config 2
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/shard2
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --sim-shards 8 --steps 3 --warmup 1 --no-cpu > $O/trace.json 2> $O/trace.err || exit 1
cd $R
for k in 8 4 2; do
  timeout -k 10 400 python -u bench.py --sim-shards $k --steps 5 --warmup 2 --no-cpu > $O/sim$k.json 2> $O/sim$k.err || exit 1
done
timeout -k 10 300 python -u bench.py --subs 1000000 --steps 20 --warmup 5 > $O/bench_config2_1m.json 2> $O/bench_config2_1m.err || exit 1
