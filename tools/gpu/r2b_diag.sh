# 100M-retained Messages diagnostic (host check, device check, image and walk), then the walk
# variants (k_walku at 6 waves/SIMD vs k_walk).
set -o pipefail
D=gpurun_out/${1:-r2b_diag}
mkdir -p $D
timeout -k 10 600 python -u tools/diag_msg.py 100000000 > $D/diag_msg.log 2>&1; echo "diag rc=$?"; cut -c1-300 $D/diag_msg.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "9=16;9=8" > $D/tune_walk.jsonl 2> $D/tune_walk.err || { echo "tune rc=$?"; tail -3 $D/tune_walk.err; exit 1; }
cat $D/tune_walk.jsonl
