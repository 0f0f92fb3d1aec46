# Round 3 (session 2): smoke (now also host span results), configs 1 and 2 on the final engine (10k and 1M subscriptions, 1M topics,
# with the CPU baseline and the end-to-end leg), and the sharded step simulated with 2/4/8
# shards at 10M.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3zi}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 300 python -u bench.py --subs 10000 > $D/bench_config1_10k.json 2> $D/bench_config1_10k.err || { echo "c1 rc=$?"; tail -5 $D/bench_config1_10k.err; exit 1; }
cut -c1-250 $D/bench_config1_10k.json
timeout -k 10 300 python -u bench.py --subs 1000000 > $D/bench_config2_1m.json 2> $D/bench_config2_1m.err || { echo "c2 rc=$?"; tail -5 $D/bench_config2_1m.err; exit 1; }
cut -c1-250 $D/bench_config2_1m.json
for S in 2 4 8; do
  timeout -k 10 420 python -u bench.py --sim-shards $S --steps 5 --warmup 2 --no-cpu > $D/bench_sim${S}_10m.json 2> $D/bench_sim${S}_10m.err || { echo "sim$S rc=$?"; tail -5 $D/bench_sim${S}_10m.err; exit 1; }
  cut -c1-250 $D/bench_sim${S}_10m.json
done
