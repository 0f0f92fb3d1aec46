# Round 3 (session 2): host span results with the sets' written patches packed (k_set_pack),
# the side stream at the greatest priority (its own hardware queue): the C++ mirror,
# the whole GPU suite, the default bench line (end_to_end), the end-to-end probe traced, and the
# set pass A/B: 2 (default), 1, 4 partner links per batch; spans copied by k_host_copy.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3zd}
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
cd $R
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --configs "18=0;18=32;18=64" --reps 3 > $D/set_ab.jsonl 2> $D/set_ab.err || { echo "ab rc=$?"; tail -5 $D/set_ab.err; exit 1; }
cut -c1-260 $D/set_ab.jsonl
