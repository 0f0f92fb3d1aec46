# Round 3 (session 2): host span results with the sets' written patches packed (k_set_pack),
# their own non-blocking stream (the spans' copy overlaps the merge kernels): the C++ mirror,
# the whole GPU suite, the default bench line (end_to_end), and the end-to-end probe traced.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3zc}
mkdir -p $D
timeout -k 5 150 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -20 $D/cpp.log; exit 1; }
tail -2 $D/cpp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
cut -c1-300 $D/bench_default.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $D/e2e_trace -o run -- python3 $R/tools/e2e_probe.py > $D/e2e_probe.jsonl 2> $D/e2e_probe.err || { echo "e2e probe rc=$?"; tail -5 $D/e2e_probe.err; exit 1; }
cut -c1-400 $D/e2e_probe.jsonl
