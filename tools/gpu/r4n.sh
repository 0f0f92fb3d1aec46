#!/bin/bash
# round 4: first-batch host results with outgrown pools (k_set_pack fix), pipelined host results,
# the C++ mirror under FIFO update locks, the pipelining diagnosis
set -o pipefail
D=gpurun_out/r4n; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "first_batch_outgrows or pipelined or host_spans or patch_pool" > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 200 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1; echo "cpp rc=$?"
grep -E "slowest|over 2 ms|longest|REQUIRE|failed" $D/cpp.log
timeout -k 10 250 python -u tools/e2e_pipe.py > $D/e2e_pipe.txt 2>&1 || { echo "e2e rc=$?"; tail -5 $D/e2e_pipe.txt; exit 1; }
timeout -k 10 250 python -u tools/e2e_pipe.py 10000000 --pinned >> $D/e2e_pipe.txt 2>&1 || { echo "e2e pinned rc=$?"; tail -5 $D/e2e_pipe.txt; exit 1; }
cat $D/e2e_pipe.txt
