# Full GPU suite, then k_merge register budget (8 vs 6 waves/SIMD) with dedup at 10M.
set -o pipefail
D=gpurun_out/${1:-r2c_suite}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "7=8;7=6" > $D/tune_10m.jsonl 2> $D/tune_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_10m.err; exit 1; }
cat $D/tune_10m.jsonl
