# Counters of the two walk variants (k_walku: 9=8; k_walk<.., false>: 9=1) on the 10M index.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r2b_walkpmc}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
T="python3 $R/tools/tune_spans.py --subs 10000000 --reps 1 --steps 2 --configs 9=8;9=1"
KR="k_walk"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "$KR" --output-format csv -d $D/sq -o run -- $T > $D/sq.log 2>&1 || { echo "sq rc=$?"; tail -3 $D/sq.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- $T > $D/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-include-regex "$KR" --output-format csv -d $D/tcc -o run -- $T > $D/tcc.log 2>&1 || { echo "tcc rc=$?"; tail -3 $D/tcc.log; }
cd $R
python profiles/summarize.py $D/sq $D/fetch $D/tcc --pmc > $D/walk_pmc.json
python - $D/walk_pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    print(k[:34], {c: round(x["per_dispatch"]) for c, x in v.items() if isinstance(x, dict) and "per_dispatch" in x})
PY
