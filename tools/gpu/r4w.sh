#!/bin/bash
# round 4: config 5's oracle side at full size (100M retained, 100k filters) on the round-4 tree:
# sample digests, counters, the fast CPU restatement's baseline (CPU only; the GPU run reads it)
set -o pipefail
D=gpurun_out/r4w; mkdir -p $D
timeout -k 10 1100 python -u bench_messages.py --retained 100000000 --oracle-only $D/msg100m_oracle.json > $D/oracle.log 2>&1 || { echo "oracle rc=$?"; tail -20 $D/oracle.log; exit 1; }
grep -v working $D/oracle.log | tail -8
python -c "import json; o=json.load(open('$D/msg100m_oracle.json')); print(o['cpu']['value'], o['cpu']['literal']['value'], o['sample_filters'])"
