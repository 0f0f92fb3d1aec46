#!/bin/bash
# round 4: config 4 at 50M with its parity sample (oracle child process, CPU baseline on); the
# 16k-topic batch line
set -o pipefail
D=gpurun_out/r4v; mkdir -p $D
timeout -k 10 300 python -u bench.py --topics 16384 --steps 50 --warmup 5 > $D/bench_16k.json 2> $D/bench_16k.err || { echo "16k rc=$?"; tail -20 $D/bench_16k.err; exit 1; }
timeout -k 10 800 python -u bench.py --mix iot --subs 50000000 --steps 10 > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; grep -v working $D/bench_iot_50m.err | tail -20; exit 1; }
python - <<'PY'
import json
for f in ("bench_16k", "bench_iot_50m"):
    b = json.loads(open(f"gpurun_out/r4v/{f}.json").read().strip().splitlines()[-1])
    ps = b.get("parity_sample", {})
    e = b.get("end_to_end", {})
    print(f, round(b["value"] / 1e6, 1), "M/s", round(b["ms_per_step"], 4), "ms", "parity", ps.get("bit_exact"), ps.get("topics"), "cpu", (b.get("cpu_baseline") or {}).get("value"), "e2e", e.get("value"), (e.get("pipelined") or {}).get("value"))
PY
