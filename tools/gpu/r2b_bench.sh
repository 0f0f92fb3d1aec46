# Round 2 artefacts: default bench line (spans, 10M, CPU baseline), the row format, 1M, and a
# rocprofv3 kernel trace of the default bench. Each step under its own time limit.
set -o pipefail
D=gpurun_out/${1:-r2b_bench}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
cat $D/bench_default.json
timeout -k 10 300 python -u bench.py --no-cpu --format rows --steps 10 --warmup 3 > $D/bench_10m_rows.json 2> $D/bench_10m_rows.err || { echo "rows rc=$?"; exit 1; }
cat $D/bench_10m_rows.json
timeout -k 10 300 python -u bench.py --subs 1000000 --steps 10 --warmup 3 > $D/bench_1m.json 2> $D/bench_1m.err || { echo "1m rc=$?"; exit 1; }
cat $D/bench_1m.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/$D/prof_bench.json 2> $GRAFT_REPO_ROOT/$D/prof_bench.err
echo "rocprof rc=$?"
