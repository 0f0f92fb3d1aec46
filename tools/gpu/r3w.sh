# Round 3 (session 2): the fused walk on 8-lane groups (32 topics per workgroup, 10 levels and 24
# gathers staged): the parity file with MQ_OPT_WALK_GROUP 8 for every index, then 16 vs 8 at 10M.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3w}
mkdir -p $D
MQ_ENGINE_OPTIONS="15=8" timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v --timeout 170 --timeout-method thread > $D/pytest_g8.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_g8.log; exit 1; }
tail -3 $D/pytest_g8.log
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "15=16;15=8" > $D/group_10m.jsonl 2> $D/group_10m.err || { echo "tune rc=$?"; tail -5 $D/group_10m.err; exit 1; }
cut -c1-600 $D/group_10m.jsonl
