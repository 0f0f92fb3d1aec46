#!/bin/bash
# round 4: the whole GPU suite on the current tree; config 4 at 50M with its parity sample (oracle
# child process, CPU baseline on); the 16k-topic batch line (the Go stage's batch size)
set -o pipefail
D=gpurun_out/r4u; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 420 python -u bench.py --mix iot --subs 50000000 --steps 10 > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -20 $D/bench_iot_50m.err; exit 1; }
timeout -k 10 300 python -u bench.py --topics 16384 --steps 50 --warmup 5 > $D/bench_16k.json 2> $D/bench_16k.err || { echo "16k rc=$?"; tail -20 $D/bench_16k.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_iot_50m", "bench_16k"):
    b = json.loads(open(f"gpurun_out/r4u/{f}.json").read().strip().splitlines()[-1])
    ps = b.get("parity_sample", {})
    print(f, round(b["value"] / 1e6, 1), "M/s", round(b["ms_per_step"], 3), "ms", "parity", ps.get("bit_exact"), ps.get("topics"), "cpu", b["cpu_baseline"]["value"] if b.get("cpu_baseline") else None)
PY
