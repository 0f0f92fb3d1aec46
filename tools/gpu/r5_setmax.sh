# Round 5: the longest merge set's phases (pair analysis vs resolution) at 16k and 1M topics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/setmax
mkdir -p $O
timeout -k 10 300 python -u bench.py --topics 16384 --steps 100 --warmup 20 --no-cpu > $O/bench_16k.json 2> $O/bench_16k.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 > $O/bench_default.json 2> $O/bench_default.err || exit 1
