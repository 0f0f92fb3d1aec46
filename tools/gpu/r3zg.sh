# Round 3 (session 2): every host topic's patch_base set on the device (k_host_rebase, no host pass
# over the records): the C++ mirror, the whole GPU suite, the end-to-end probe and the bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3zg}
mkdir -p $D
timeout -k 5 150 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -20 $D/cpp.log; exit 1; }
tail -1 $D/cpp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 300 python -u tools/e2e_probe.py > $D/e2e_probe.jsonl 2> $D/e2e_probe.err || { echo "probe rc=$?"; tail -5 $D/e2e_probe.err; exit 1; }
cut -c1-200 $D/e2e_probe.jsonl
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
cut -c1-300 $D/bench_default.json
