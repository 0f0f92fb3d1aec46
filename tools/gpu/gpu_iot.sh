# Config 4 (IoT fan-in) at one-GPU scale: 50M exact device filters + 1% dashboards, 1M device
# topics per step; then the headline bench's host-memory footprint (for the 8-rank run).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/iot
mkdir -p $D
timeout -k 10 900 python bench.py --mix iot --subs 50000000 --steps 5 --warmup 2 --no-cpu > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || exit 1
