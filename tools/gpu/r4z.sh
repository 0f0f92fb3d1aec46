#!/bin/bash
# round 4: the edge table at 1/8 by default: headline bench line (CPU baseline, parity sample),
# config 4 at 50M, config 2 at 1M, then the whole GPU suite
set -o pipefail
D=gpurun_out/r4z; mkdir -p $D
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -20 $D/bench_default.err; exit 1; }
timeout -k 10 300 python -u bench.py --mix iot --subs 50000000 --steps 10 --no-cpu > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -20 $D/bench_iot_50m.err; exit 1; }
timeout -k 10 300 python -u bench.py --subs 1000000 > $D/bench_config2_1m.json 2> $D/bench_config2_1m.err || { echo "c2 rc=$?"; tail -20 $D/bench_config2_1m.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_default", "bench_iot_50m", "bench_config2_1m"):
    b = json.loads(open(f"gpurun_out/r4z/{f}.json").read().strip().splitlines()[-1])
    k = b.get("kernels_ms_per_step") or {}
    e = b.get("end_to_end") or {}
    print(f, round(b["value"] / 1e6, 1), "M/s", round(b["ms_per_step"], 3), {a: round(v, 3) for a, v in k.items()}, "parity", (b.get("parity_sample") or {}).get("bit_exact"), "frac", b["roofline"]["frac"], "cpu", (b.get("cpu_baseline") or {}).get("value"), "pipelined", (e.get("pipelined") or {}).get("value"))
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
