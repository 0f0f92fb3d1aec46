# Round 2: patch regions (one counter per region) — GPU suite, k_merge variants, PMC pass.
# PMC pass of instruction counters on the 1M span-format run.
set -o pipefail
D=gpurun_out/r2_tune4
mkdir -p $D
export TMPDIR=/tmp
rocprofv3 -L > $D/counters.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
echo "pytest rc=$?" | tee -a $D/pytest_gpu.log
tail -3 $D/pytest_gpu.log
timeout -k 10 400 python tools/tune_spans.py --subs 10000000 --reps 2 --configs "7=1;7=8" > $D/tune_10m.jsonl 2> $D/tune_10m.err || exit 1
cat $D/tune_10m.jsonl
timeout -k 10 300 python tools/tune_spans.py --subs 1000000 --reps 2 --configs "7=1;7=8" > $D/tune_1m.jsonl 2> $D/tune_1m.err || exit 1
cat $D/tune_1m.jsonl
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -d $GRAFT_REPO_ROOT/$D/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/tools/tune_spans.py --subs 1000000 --reps 1 --steps 2 --configs "7=1" > $GRAFT_REPO_ROOT/$D/pmc1.out 2>&1
echo "pmc rc=$?"
