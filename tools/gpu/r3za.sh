# Round 3 (session 2): host span results with merge-set patches (ABI v7). Standalone C++ mirror
# test (SubscribersBatch reads host results), smoke, the whole GPU suite, the default bench line
# (its end_to_end leg: spans through host memory on the whole batch), then the set pass's early
# stop A/B (MQ_OPT_SET_EXP bit 4 turns it off) and the link prefetch (bit 5) on the same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3za}
mkdir -p $D
timeout -k 5 150 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -20 $D/cpp.log; exit 1; }
tail -3 $D/cpp.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -60 $D/pytest_gpu.log; exit 1; }
tail -3 $D/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
cut -c1-600 $D/bench_default.json
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --configs "18=0,7=8;18=16,7=8;18=32,7=8;18=32,7=6" --reps 3 > $D/early_stop_ab.jsonl 2> $D/early_stop_ab.err || { echo "ab rc=$?"; tail -5 $D/early_stop_ab.err; exit 1; }
cut -c1-300 $D/early_stop_ab.jsonl
