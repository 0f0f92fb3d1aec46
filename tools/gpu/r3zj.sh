# Round 3 (session 2), short: smoke (now also host span results), config 2 (1M subscriptions, with
# the CPU baseline and the end-to-end leg) and the 8-shard simulation at 10M on the final engine.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3zj}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 300 python -u bench.py --subs 1000000 > $D/bench_config2_1m.json 2> $D/bench_config2_1m.err || { echo "c2 rc=$?"; tail -5 $D/bench_config2_1m.err; exit 1; }
cut -c1-250 $D/bench_config2_1m.json
timeout -k 10 420 python -u bench.py --sim-shards 8 --steps 5 --warmup 2 --no-cpu > $D/bench_sim8_10m.json 2> $D/bench_sim8_10m.err || { echo "sim8 rc=$?"; tail -5 $D/bench_sim8_10m.err; exit 1; }
cut -c1-250 $D/bench_sim8_10m.json
