#!/bin/bash
# round 4: Messages literal lookups in the image's own edge table: parity, then 10M A/B
set -o pipefail
D=gpurun_out/r4x; mkdir -p $D
timeout -k 10 200 python -u -c "import torch; print('torch', torch.__version__, flush=True)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 60 --timeout-method thread -k "messages or retained" > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 500 python -u bench_messages.py > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -20 $D/msg_10m.err; exit 1; }
timeout -k 10 300 python -u bench_messages.py --no-cpu --no-img-edges > $D/msg_10m_noedges.json 2> $D/msg_10m_noedges.err || { echo "msg2 rc=$?"; tail -20 $D/msg_10m_noedges.err; exit 1; }
python - <<'PY'
import json
for f in ("msg_10m", "msg_10m_noedges"):
    b = json.loads(open(f"gpurun_out/r4x/{f}.json").read().strip().splitlines()[-1])
    print(f, round(b["value"] / 1e6, 2), "M/s", round(b["ms_per_step"], 3), {k: round(v, 3) for k, v in b["kernels_ms_per_step"].items()}, b.get("image_build_ms"))
PY
