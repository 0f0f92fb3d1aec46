#!/bin/bash
# round 4: the Messages line at 10M retained with its PMC traffic (pmc_traffic.json) and parity sample
set -o pipefail
D=gpurun_out/r4msgf; mkdir -p $D
timeout -k 10 500 python -u bench_messages.py > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -20 $D/msg_10m.err; exit 1; }
python -c "
import json; b=json.loads(open('$D/msg_10m.json').read().strip().splitlines()[-1])
print(round(b['value']/1e6,2), round(b['ms_per_step'],3), b['parity_sample'], b['cpu_baseline']['value'], {k: (round(v,3) if isinstance(v,float) else v) for k,v in b['roofline'].items() if k in ('frac','traffic','hbm_traffic_GBps','hbm_traffic_frac')})"
