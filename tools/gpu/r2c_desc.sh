# k_desc_g16 (16 lanes per topic): parity file + headline-scale parity, then the span step at 10M.
set -o pipefail
D=gpurun_out/${1:-r2c_desc}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $D/parity.log; exit 1; }
tail -1 $D/parity.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 400 --timeout-method thread > $D/scale.log 2>&1 || { echo "scale rc=$?"; tail -20 $D/scale.log; exit 1; }
tail -1 $D/scale.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "12=1;12=0" > $D/tune_10m.jsonl 2> $D/tune_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_10m.err; exit 1; }
cat $D/tune_10m.jsonl
