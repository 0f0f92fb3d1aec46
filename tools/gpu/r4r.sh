#!/bin/bash
# round 4: host and copy streams created together (distinct hardware queues); bench pipelined leg
set -o pipefail
D=gpurun_out/r4r; mkdir -p $D
MQ_TRACE_SUBMIT=1 timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -20 $D/bench_default.err; exit 1; }
python - <<'PY'
import json
b = json.loads(open("gpurun_out/r4r/bench_default.json").read().strip().splitlines()[-1])
e = b["end_to_end"]
print(round(b["value"] / 1e6, 1), "M/s", "e2e", round(e["value"] / 1e6, 1), "pipelined", round(e["pipelined"]["value"] / 1e6, 1), e["pipelined"]["runs_ms"], e["pipelined"]["median_run_submit_wait_ms"])
PY
grep mq_match_spans_submit $D/bench_default.err | tail -12
