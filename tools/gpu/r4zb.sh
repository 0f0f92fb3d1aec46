#!/bin/bash
# round 4: the edge table at 1/16 by default: headline bench line (CPU baseline, parity sample),
# config 2 at 1M, Messages at 10M retained, then the whole GPU suite
set -o pipefail
D=gpurun_out/r4zb; mkdir -p $D
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -20 $D/bench_default.err; exit 1; }
timeout -k 10 300 python -u bench.py --subs 1000000 > $D/bench_config2_1m.json 2> $D/bench_config2_1m.err || { echo "c2 rc=$?"; tail -20 $D/bench_config2_1m.err; exit 1; }
timeout -k 10 300 python -u bench_messages.py --no-cpu > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -20 $D/msg_10m.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_default", "bench_config2_1m", "msg_10m"):
    b = json.loads(open(f"gpurun_out/r4zb/{f}.json").read().strip().splitlines()[-1])
    k = b.get("kernels_ms_per_step") or {}
    e = b.get("end_to_end") or {}
    print(f, round(b["value"] / 1e6, 1), "M/s", round(b["ms_per_step"], 3), {a: round(v, 3) for a, v in k.items()}, "parity", (b.get("parity_sample") or {}).get("bit_exact"), "frac", (b.get("roofline") or {}).get("frac"), "cpu", (b.get("cpu_baseline") or {}).get("value"), "pipelined", (e.get("pipelined") or {}).get("value"))
PY
grep "peak host memory" $D/bench_default.err | tail -1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/pytest.log 2>&1; echo "pytest rc=$?"
tail -2 $D/pytest.log
