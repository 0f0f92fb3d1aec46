#!/bin/bash
# round 4 final tree: config 4 at 50M with its parity sample (oracle child process) and CPU baseline
set -o pipefail
D=gpurun_out/r4iot; mkdir -p $D
timeout -k 10 800 python -u bench.py --mix iot --subs 50000000 --steps 10 > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; grep -v working $D/bench_iot_50m.err | tail -20; exit 1; }
python -c "
import json; b=json.loads(open('$D/bench_iot_50m.json').read().strip().splitlines()[-1])
print(round(b['value']/1e6,1), round(b['ms_per_step'],4), b['parity_sample'].get('bit_exact'), b['parity_sample'].get('topics'), b['cpu_baseline']['value'])"
grep -v working $D/bench_iot_50m.err | grep -E "index built|peak host" | cut -c1-200
