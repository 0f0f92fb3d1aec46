#!/bin/bash
# round 4: slab-carved pinned blocks + FIFO locks (C++ mirror update latency); bench default line
# with 8-batch pipelined runs
set -o pipefail
D=gpurun_out/r4o; mkdir -p $D
timeout -k 10 200 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1; echo "cpp rc=$?"
grep -E "slowest|over 2 ms|longest|REQUIRE|failed" $D/cpp.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "host_spans or pipelined or patch_pool or device_matches_host" > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -20 $D/bench_default.err; exit 1; }
python - <<'PY'
import json
b = json.loads(open("gpurun_out/r4o/bench_default.json").read().strip().splitlines()[-1])
e = b["end_to_end"]
print(round(b["value"] / 1e6, 1), "M/s", b["ms_per_step"], "e2e", round(e["value"] / 1e6, 1), "pipelined", round(e["pipelined"]["value"] / 1e6, 1), e["pipelined"]["runs_ms"], e["pipelined"]["bytes_per_topic"])
PY
