# Iteration: GPU suite, then the 10M and 1M span-format bench lines (no CPU baseline).
set -o pipefail
D=gpurun_out/${1:-r2b_iter}
mkdir -p $D
bash tools/gpu/r2_suite.sh ${1:-r2b_iter} || exit 1
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_10m.json 2> $D/bench_10m.err || { echo "bench rc=$?"; tail -5 $D/bench_10m.err; exit 1; }
python tools/show.py $D/bench_10m.json
timeout -k 10 300 python -u bench.py --subs 1000000 --no-cpu > $D/bench_1m.json 2> $D/bench_1m.err || { echo "1m rc=$?"; exit 1; }
python tools/show.py $D/bench_1m.json
