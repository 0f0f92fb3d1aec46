#!/bin/bash
# round 4: where the bench's pipelined batches spend their time, beside the standalone diagnosis
set -o pipefail
D=gpurun_out/r4p; mkdir -p $D
timeout -k 10 250 python -u tools/e2e_pipe.py 10000000 --expected > $D/e2e_pipe.txt 2>&1 || { echo "e2e rc=$?"; tail -5 $D/e2e_pipe.txt; exit 1; }
cat $D/e2e_pipe.txt | cut -c1-900
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -20 $D/bench_default.err; exit 1; }
python - <<'PY'
import json
b = json.loads(open("gpurun_out/r4p/bench_default.json").read().strip().splitlines()[-1])
e = b["end_to_end"]
print(round(b["value"] / 1e6, 1), "M/s", "e2e", round(e["value"] / 1e6, 1), "pipelined", round(e["pipelined"]["value"] / 1e6, 1), e["pipelined"]["runs_ms"], e["pipelined"]["median_run_submit_wait_ms"])
PY
