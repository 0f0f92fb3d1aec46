# Last evidence on the final tree (heavy-first set list): smoke, full GPU suite, span step at
# 10M, default bench line.
set -o pipefail
D=gpurun_out/${1:-r2c_last2}
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "14=1;14=0" > $D/tune_10m.jsonl 2> $D/tune_10m.err || { echo "tune rc=$?"; tail -5 $D/tune_10m.err; exit 1; }
cat $D/tune_10m.jsonl
timeout -k 10 600 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
python tools/show.py $D/bench_default.json
python -c "import json;d=json.load(open('$D/bench_default.json'));print(d['roofline']['frac'], d['roofline']['traffic'], d['parity_sample'])"
