#!/bin/bash
# round 4: Messages PMC traffic at 10M retained (the image's edge table, one-sync batches):
# FETCH_SIZE and WRITE_SIZE in separate passes of bench_messages.py
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r4mp; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_msgq|k_msg_copy"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- python3 $R/bench_messages.py $ARGS > $D/fetch.json 2> $D/fetch.err || { echo "fetch rc=$?"; tail -5 $D/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/write -o run -- python3 $R/bench_messages.py $ARGS > $D/write.json 2> $D/write.err || { echo "write rc=$?"; tail -5 $D/write.err; exit 1; }
cd $R
python profiles/summarize.py $D/fetch $D/write --pmc > $D/pmc.json
python - <<'PY'
import json
p = json.load(open("gpurun_out/r4mp/pmc.json"))
for k, v in p.items():
    print(k, {a: round(b / 1e6, 1) for a, b in v["hbm_bytes_per_dispatch"].items()}, v["FETCH_SIZE"]["dispatches"])
PY
