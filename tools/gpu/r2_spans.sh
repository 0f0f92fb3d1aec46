# Round 2: first span-format check — GPU test suite, then 10M bench in both formats, a 1M bench,
# and a rocprofv3 kernel trace of the 10M span-format bench.
set -o pipefail
D=gpurun_out/r2_spans
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a $D/pytest_gpu.log
tail -5 $D/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu > $D/bench_10m_spans.json 2> $D/bench_10m_spans.err || exit 1
cat $D/bench_10m_spans.json
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu --format rows > $D/bench_10m_rows.json 2> $D/bench_10m_rows.err || exit 1
cat $D/bench_10m_rows.json
timeout -k 10 300 python bench.py --subs 1000000 --steps 10 --warmup 3 --no-cpu > $D/bench_1m_spans.json 2> $D/bench_1m_spans.err || exit 1
cat $D/bench_1m_spans.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/$D/prof_bench.json 2> $GRAFT_REPO_ROOT/$D/prof_bench.err
echo "rocprof rc=$?"
