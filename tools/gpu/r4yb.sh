#!/bin/bash
# round 4: the subscription edge table at 1/16 load against 1/8 (the default)
set -o pipefail
D=gpurun_out/r4yb; mkdir -p $D
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_load8.json 2> $D/bench_load8.err || { echo "b8 rc=$?"; tail -20 $D/bench_load8.err; exit 1; }
MQ_ENGINE_OPTIONS=13=16 timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_load16.json 2> $D/bench_load16.err || { echo "b16 rc=$?"; tail -20 $D/bench_load16.err; exit 1; }
python - <<'PY'
import json
for f in ("bench_load8", "bench_load16"):
    b = json.loads(open(f"gpurun_out/r4yb/{f}.json").read().strip().splitlines()[-1])
    k = b.get("kernels_ms_per_step") or {}
    print(f, round(b["value"] / 1e6, 1), "M/s", round(b["ms_per_step"], 3), {a: round(v, 3) for a, v in k.items()}, b["roofline"]["frac"])
PY
grep "engine index built" $D/bench_load16.err | cut -c1-220
