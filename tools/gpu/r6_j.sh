#!/bin/bash
# Round 6: (1) the Messages key index (parity: every Messages test; the 10M line); (2) the C++
# mirror's concurrent test, three times, MQ_SLOW_MS milestones; (3) the north star's LDS staging
# bounded by attribution (development library: levels 0 / 0-1 looked up ahead of the walk)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "messages" tests/test_gpu_scale.py::test_messages_10m_retained_100k_filters -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_msg.log 2>&1 || { tail -30 $O/pytest_msg.log; exit 1; }
timeout -k 10 300 python -u bench_messages.py --steps 10 --warmup 3 --no-cpu > $O/msg_10m.json 2> $O/msg_10m.err || { tail -20 $O/msg_10m.err; exit 1; }
for k in 1 2 3; do
  MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp$k.out 2> $O/cpp$k.err
  echo "cpp run $k rc=$?"
done
MQ_LIB_DIR=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_dev timeout -k 10 400 python -u tools/ab_options.py --check 4096 --variants 24=0 24=1 24=2 --rounds 3 > $O/ab_hint.json 2> $O/ab_hint.err || exit 1
