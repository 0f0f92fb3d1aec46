# Round 3, first GPU pass: the C++ host mirror's tests standalone (writer-preferring handle
# lock), frontier walk vs thread-per-topic walk at 10M, then the GPU suite (frontier walk default).
set -o pipefail
D=gpurun_out/${1:-r3a}
mkdir -p $D
timeout -k 5 120 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -20 $D/cpp.log; exit 1; }
tail -3 $D/cpp.log
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "15=0;15=16;15=8;15=4" > $D/tune_walk_10m.jsonl 2> $D/tune_walk_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_walk_10m.err; exit 1; }
cat $D/tune_walk_10m.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -3 $D/pytest_gpu.log
