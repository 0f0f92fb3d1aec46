# Round 3 (session 2): k_desc fused into the frontier walk's epilogue (MQ_OPT_FUSE_DESC 17):
# parity (the span / dedup / one-sync tests and smoke), then the 10M step fused vs not.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3m}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
cat $D/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 170 --timeout-method thread > $D/pytest_parity.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_parity.log; exit 1; }
tail -3 $D/pytest_parity.log
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "17=1;17=0" > $D/fuse_10m.jsonl 2> $D/fuse_10m.err || { echo "tune rc=$?"; tail -5 $D/fuse_10m.err; exit 1; }
cut -c1-600 $D/fuse_10m.jsonl
