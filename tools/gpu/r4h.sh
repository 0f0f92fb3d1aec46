# Round 4: copy-on-write against live host span results (updates no longer wait for results):
# the liveness/parity tests, the C++ concurrency test (slowest update), smoke.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4h}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread -k "survives_updates or random_small or incremental or long_lists or many_merging or partner_map or cpp_host" > $D/pytest_cow.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_cow.log; exit 1; }
tail -2 $D/pytest_cow.log
timeout -k 10 300 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -30 $D/cpp.log; exit 1; }
grep -E "slowest|passed|FAIL" $D/cpp.log
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --ignore tests/test_gpu_scale.py --timeout 170 --timeout-method thread > $D/pytest_all.log 2>&1 || { echo "pytest all rc=$?"; tail -40 $D/pytest_all.log; exit 1; }
tail -2 $D/pytest_all.log
