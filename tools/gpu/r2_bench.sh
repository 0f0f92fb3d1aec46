# Round 2: GPU suite, then the default bench line (span format, 10M, CPU baseline) and the
# k_merge variants once more.
set -o pipefail
D=gpurun_out/${1:-r2_bench}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a $D/pytest_gpu.log
tail -3 $D/pytest_gpu.log
timeout -k 10 600 python bench.py > $D/bench_default.json 2> $D/bench_default.err || exit 1
cat $D/bench_default.json
timeout -k 10 400 python tools/tune_spans.py --subs 10000000 --reps 2 --configs "7=1;7=6;7=8" > $D/tune_10m.jsonl 2> $D/tune_10m.err || exit 1
cat $D/tune_10m.jsonl
