# Set-shared patches in device results (ABI v6, dedup on by default): GPU parity file, span step
# with dedup on/off at 10M, then the default bench line (parity sample from the timed result).
set -o pipefail
D=gpurun_out/${1:-r2c_ref}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $D/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $D/parity.log; exit 1; }
tail -2 $D/parity.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "12=1;12=0" > $D/tune_10m.jsonl 2> $D/tune_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_10m.err; exit 1; }
cat $D/tune_10m.jsonl
timeout -k 10 600 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
python tools/show.py $D/bench_default.json
python -c "import json;d=json.load(open('$D/bench_default.json'));print(d.get('parity_sample'), d.get('roofline'), d.get('merge_work_per_topic'))"
