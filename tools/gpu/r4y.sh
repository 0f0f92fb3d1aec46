#!/bin/bash
# round 4: the subscription edge table at 1/8 load (MQ_OPT_EDGE_LOAD 8) against 1/4 (the default)
set -o pipefail
D=gpurun_out/r4y; mkdir -p $D
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_load4.json 2> $D/bench_load4.err || { echo "b4 rc=$?"; tail -20 $D/bench_load4.err; exit 1; }
MQ_ENGINE_OPTIONS=13=8 timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_load8.json 2> $D/bench_load8.err || { echo "b8 rc=$?"; tail -20 $D/bench_load8.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_load4", "bench_load8"):
    b = json.loads(open(f"gpurun_out/r4y/{f}.json").read().strip().splitlines()[-1])
    k = b.get("kernels_ms_per_step") or {}
    print(f, round(b["value"] / 1e6, 1), "M/s", round(b["ms_per_step"], 3), {a: round(v, 3) for a, v in k.items()} if isinstance(k, dict) else k, b["parity_sample"].get("bit_exact"), b["roofline"]["frac"])
PY
