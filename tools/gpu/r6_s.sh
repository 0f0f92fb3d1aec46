#!/bin/bash
# Round 6: where a 16k-topic host-results call spends its 0.53 ms — tools/latency.cpp at 10M with
# MQ_SLOW_MS milestones on every call over 0.3 ms
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/s
mkdir -p $O
( while true; do date >> $O/heartbeat.log; sleep 60; done ) &
HB=$!
trap "kill $HB" EXIT
MQ_SLOW_MS=0.3 timeout -k 10 400 mqtt-server_amd/build/latency 10000000 1 > $O/latency.jsonl 2> $O/latency.err || exit 1
