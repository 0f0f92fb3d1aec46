# k_merge register budget with the set pass compiled apart: 8 vs 6 waves per SIMD at 10M and 1M.
set -o pipefail
D=gpurun_out/${1:-r2c_wpe}
mkdir -p $D
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "7=8;7=6" > $D/tune_10m.jsonl 2> $D/tune_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_10m.err; exit 1; }
cat $D/tune_10m.jsonl
timeout -k 10 200 python -u tools/tune_spans.py --subs 1000000 --reps 2 --configs "7=8;7=6" > $D/tune_1m.jsonl 2> $D/tune_1m.err || { echo "tune rc=$?"; exit 1; }
cat $D/tune_1m.jsonl
