# Counters: the available counter list, then SQ occupancy / stall counters of the span step's
# kernels (one pass per counter group), and the bench line of the current tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r2b_sq}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $D/counters_avail.txt 2>&1 || echo "list rc=$?"
ARGS="--steps 2 --warmup 1 --no-cpu"
KR="k_walk|k_merge|k_desc"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$KR" --output-format csv -d $D/sq1 -o run -- python3 $R/bench.py $ARGS > $D/sq1.json 2> $D/sq1.err || { echo "sq1 rc=$?"; tail -3 $D/sq1.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES --kernel-include-regex "$KR" --output-format csv -d $D/sq2 -o run -- python3 $R/bench.py $ARGS > $D/sq2.json 2> $D/sq2.err || { echo "sq2 rc=$?"; tail -3 $D/sq2.err; }
cd $R
python profiles/summarize.py $D/sq1 $D/sq2 --pmc > $D/sq.json
python - $D/sq.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    print(k[:40], {c: round(x["per_dispatch"]) for c, x in v.items() if isinstance(x, dict) and "per_dispatch" in x})
PY
timeout -k 10 300 python -u bench.py --no-cpu > $D/bench_10m.json 2> $D/bench_10m.err || { echo "bench rc=$?"; exit 1; }
python tools/show.py $D/bench_10m.json
