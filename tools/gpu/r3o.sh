# Round 3 (session 2): flattened partner-link resolution in k_merge (kFlatU links per lane in
# flight): smoke, the span/merge parity tests, the 10M step.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3o}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -x -v --timeout 170 --timeout-method thread > $D/pytest_parity.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_parity.log; exit 1; }
tail -3 $D/pytest_parity.log
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "17=1;17=0" --work > $D/flat_10m.jsonl 2> $D/flat_10m.err || { echo "tune rc=$?"; tail -5 $D/flat_10m.err; exit 1; }
cut -c1-900 $D/flat_10m.jsonl
