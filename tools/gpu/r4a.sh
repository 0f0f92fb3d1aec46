# Round 4: the new scale tests (10M unsharded through the timed path, 10M over 8 shards, 10M
# retained x 100k filters), smoke, and the default bench line with its oracle side in a child
# process.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4a}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 600 --timeout-method thread > $D/pytest_scale.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_scale.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $D/pytest_scale.log | tail -8
timeout -k 10 600 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
cut -c1-400 $D/bench_default.json
