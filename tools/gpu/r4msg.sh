#!/bin/bash
# round 4: the Messages export threshold (MQ_OPT_MSG_EXPORT) with the image's edge table
set -o pipefail
D=gpurun_out/r4msg; mkdir -p $D
for t in 256 1024 2048; do
  MQ_ENGINE_OPTIONS=19=$t timeout -k 10 300 python -u bench_messages.py --no-cpu > $D/msg_exp$t.json 2> $D/msg_exp$t.err || { echo "msg $t rc=$?"; tail -20 $D/msg_exp$t.err; exit 1; }
  python -c "
import json; b=json.loads(open('$D/msg_exp$t.json').read().strip().splitlines()[-1])
print($t, round(b['value']/1e6,2), round(b['ms_per_step'],3), {k: round(v,3) for k,v in b['kernels_ms_per_step'].items()})"
done
