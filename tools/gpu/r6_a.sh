#!/bin/bash
# Round 6: config 4 re-pinned on this tree — the IoT index at half edge-table load (the 50M
# index's probe regime) against the oracle, then the 50M IoT bench line with its oracle side on
# (20k-topic parity sample, roofline, CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/a
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -k "iot" -m gpu -x -v --timeout 450 --timeout-method thread > $O/pytest_iot.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --mix iot --subs 50000000 --steps 10 --warmup 3 > $O/bench_iot_50m.json 2> $O/bench_iot_50m.err || exit 1
