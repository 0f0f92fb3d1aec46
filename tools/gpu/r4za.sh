#!/bin/bash
# round 4: the whole GPU suite (the C++ mirror's readers warmed per thread)
set -o pipefail
D=gpurun_out/r4za; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $D/pytest.log 2>&1; echo "pytest rc=$?"
tail -3 $D/pytest.log
grep -E "slowest|over 2 ms|longest" $D/pytest.log | head -5
timeout -k 10 100 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1; echo "cpp rc=$?"
grep -E "slowest|over 2 ms|longest|failed" $D/cpp.log
