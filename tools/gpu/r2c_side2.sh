# Config 2 (1M subs) and config 1 (10k subs) on the final tree.
set -o pipefail
D=gpurun_out/${1:-r2c_side2}
mkdir -p $D
timeout -k 10 400 python -u bench.py --subs 1000000 > $D/bench_1m.json 2> $D/bench_1m.err || { echo "1m rc=$?"; tail -5 $D/bench_1m.err; exit 1; }
python tools/show.py $D/bench_1m.json
timeout -k 10 400 python -u bench.py --subs 10000 > $D/bench_config1_10k.json 2> $D/bench_config1_10k.err || { echo "10k rc=$?"; tail -5 $D/bench_config1_10k.err; exit 1; }
python tools/show.py $D/bench_config1_10k.json
