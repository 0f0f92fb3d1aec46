# Config 4 (IoT fan-in, 50M subscriptions, 1M device topics per step) on one GPU, with its CPU
# baseline and parity sample.
set -o pipefail
D=gpurun_out/${1:-r2c_iot}
mkdir -p $D
timeout -k 10 1000 python -u bench.py --mix iot --subs 50000000 > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -5 $D/bench_iot_50m.err; exit 1; }
python tools/show.py $D/bench_iot_50m.json
python -c "import json;d=json.load(open('$D/bench_iot_50m.json'));print(d.get('parity_sample'), d.get('roofline'), d.get('cpu_baseline'))"
