#!/bin/bash
# Round 6: the C++ mirror's concurrent test, three times, with MQ_SLOW_MS milestones (diagnosis of
# the stall right after the readers' cold first matches)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/j
mkdir -p $O
for k in 1 2 3; do
  MQ_SLOW_MS=1 timeout -k 10 120 mqtt-server_amd/build/test_topics_index > $O/cpp$k.out 2> $O/cpp$k.err
  echo "run $k rc=$?"
done
MQ_LIB_DIR=$GRAFT_REPO_ROOT/mqtt-server_amd/lib_dev timeout -k 10 400 python -u tools/ab_options.py --check 4096 --variants 24=0 24=1 24=2 --rounds 3 > $O/ab_hint.json 2> $O/ab_hint.err || exit 1
