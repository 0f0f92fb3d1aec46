# Round 3 (session 2): set pass variants A/B on one box — 2 links per batch at 8 waves per SIMD
# (default), 3 links, 7 and 6 waves per SIMD — after their parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3zh}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "set_pass_variants" -x -v --timeout 170 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 400 python -u tools/tune_spans.py --subs 10000000 --configs "18=0,7=8;18=32,7=8;18=0,7=7;18=0,7=6" --reps 3 > $D/set_ab.jsonl 2> $D/set_ab.err || { echo "ab rc=$?"; tail -5 $D/set_ab.err; exit 1; }
cut -c1-220 $D/set_ab.jsonl
