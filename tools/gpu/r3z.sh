# Round 3 (session 2): walk trials (frontier + fused desc vs thread per topic, per index size):
# smoke, the parity file, the 10M default bench step and config 4 (50M IoT) with the default.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3z}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_scale.py -x -q --timeout 170 --timeout-method thread > $D/pytest_parity.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_parity.log; exit 1; }
tail -2 $D/pytest_parity.log
timeout -k 10 400 python -u bench.py --no-cpu > $D/bench_10m.json 2> $D/bench_10m.err || { echo "bench rc=$?"; tail -5 $D/bench_10m.err; exit 1; }
cut -c1-700 $D/bench_10m.json
timeout -k 10 400 python -u bench.py --mix iot --subs 50000000 --no-cpu > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -5 $D/bench_iot_50m.err; exit 1; }
cut -c1-700 $D/bench_iot_50m.json
