# Round 3 (session 2): where the merge set pass spends its time — phase clocks (MQ_PROF_WORK)
# and SQ counters of k_merge's set pass; the batching stage with 64 submission queues.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3l}
mkdir -p $D
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 1 --configs "9=8" --work > $D/work_10m.jsonl 2> $D/work_10m.err || { echo "work rc=$?"; tail -5 $D/work_10m.err; exit 1; }
cut -c1-1500 $D/work_10m.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1 || true
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_merge|k_walkf|k_desc"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "$KR" --output-format csv -d $D/sq1 -o run -- python3 $R/bench.py $ARGS > $D/sq1.json 2> $D/sq1.err || { echo "sq1 rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/sq1 --pmc > $D/sq1_pmc.json
head -c 3000 $D/sq1_pmc.json
timeout -k 10 300 mqtt-server_amd/build/latency 10000000 3 > $D/latency_10m.jsonl 2> $D/latency_10m.err || { echo "latency rc=$?"; tail -5 $D/latency_10m.err; exit 1; }
cut -c1-420 $D/latency_10m.jsonl
grep -o "SQ_[A-Z_0-9]*" $D/counters.txt | sort -u | tr '\n' ' ' | head -c 4000
