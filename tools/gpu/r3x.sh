# Round 3 (session 2): k_dedup_insert folded into the fused walk's epilogue: smoke, the parity
# file (16- and 8-lane groups), the 10M step.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3x}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread > $D/pytest_parity.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_parity.log; exit 1; }
tail -2 $D/pytest_parity.log
MQ_ENGINE_OPTIONS="15=8" timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 170 --timeout-method thread -k "spans or one_sync or walk or merg or pair" > $D/pytest_parity_g8.log 2>&1 || { echo "pytest g8 rc=$?"; tail -40 $D/pytest_parity_g8.log; exit 1; }
tail -2 $D/pytest_parity_g8.log
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "15=16;15=8" > $D/step_10m.jsonl 2> $D/step_10m.err || { echo "tune rc=$?"; tail -5 $D/step_10m.err; exit 1; }
cut -c1-600 $D/step_10m.jsonl
