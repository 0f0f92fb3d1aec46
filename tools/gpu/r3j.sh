# Round 3 (session 2): the tree after in-place merge-record updates. Standalone C++ mirror test,
# smoke, the whole GPU suite, the default bench line with a kernel trace, then the batching stage
# (64 submitters) and the sharded step simulated with 2/4/8 shards at 10M.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3j}
mkdir -p $D
timeout -k 5 150 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -20 $D/cpp.log; exit 1; }
tail -3 $D/cpp.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $D/pytest_gpu.log; exit 1; }
tail -3 $D/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
cut -c1-1500 $D/bench_default.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $D/trace.json 2> $D/trace.err || { echo "trace rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/trace > $D/kernel_stats.json
head -c 1200 $D/kernel_stats.json
timeout -k 10 300 mqtt-server_amd/build/latency 10000000 3 > $D/latency_10m.jsonl 2> $D/latency_10m.err || { echo "latency rc=$?"; tail -5 $D/latency_10m.err; exit 1; }
cut -c1-400 $D/latency_10m.jsonl
for S in 2 4 8; do
  timeout -k 10 420 python -u bench.py --sim-shards $S --steps 5 --warmup 2 --no-cpu > $D/bench_sim${S}_10m.json 2> $D/bench_sim${S}_10m.err || { echo "sim$S rc=$?"; tail -5 $D/bench_sim${S}_10m.err; exit 1; }
  cut -c1-1200 $D/bench_sim${S}_10m.json
done
