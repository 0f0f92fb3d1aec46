# Round 3 (session 2): k_dedup_insert folded into the fused walk (smoke, parity, 10M step), the
# Messages line with the fast CPU baseline, and config 4 (50M IoT) with the frontier walk (default)
# against the thread-per-topic walk (MQ_OPT_WALK_GROUP 0).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3y}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -x -q --timeout 170 --timeout-method thread > $D/pytest_parity.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_parity.log; exit 1; }
tail -2 $D/pytest_parity.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "17=1" > $D/step_10m.jsonl 2> $D/step_10m.err || { echo "tune rc=$?"; tail -5 $D/step_10m.err; exit 1; }
cut -c1-500 $D/step_10m.jsonl
timeout -k 10 400 python -u bench_messages.py --retained 10000000 > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -5 $D/msg_10m.err; exit 1; }
cut -c1-300 $D/msg_10m.json
MQ_ENGINE_OPTIONS="15=0" timeout -k 10 400 python -u bench.py --mix iot --subs 50000000 --no-cpu > $D/bench_iot_50m_g0.json 2> $D/bench_iot_50m_g0.err || { echo "iot0 rc=$?"; tail -5 $D/bench_iot_50m_g0.err; exit 1; }
cut -c1-600 $D/bench_iot_50m_g0.json
