#!/bin/bash
# round 4: one-sync host batches read their counts through k_readback (no small copies behind the
# previous batch's result copy); host-result parity, then the bench's pipelined leg traced
set -o pipefail
D=gpurun_out/r4t; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "host_spans or pipelined or patch_pool or device_matches_host or first_batch" > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
MQ_TRACE_SUBMIT=1 timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -20 $D/bench_default.err; exit 1; }
python - <<'PY'
import json
b = json.loads(open("gpurun_out/r4t/bench_default.json").read().strip().splitlines()[-1])
e = b["end_to_end"]
print(round(b["value"] / 1e6, 1), "M/s", "e2e", round(e["value"] / 1e6, 1), "pipelined", round(e["pipelined"]["value"] / 1e6, 1), e["pipelined"]["runs_ms"], e["pipelined"]["median_run_submit_wait_ms"], "parity", b["parity_sample"]["equal"] if "equal" in b["parity_sample"] else b["parity_sample"])
PY
grep mq_match_spans_submit $D/bench_default.err | tail -6
