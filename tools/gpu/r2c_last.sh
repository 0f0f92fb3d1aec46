# Last evidence on the final tree: smoke, full GPU suite, default bench line.
set -o pipefail
D=gpurun_out/${1:-r2c_last}
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
python tools/show.py $D/bench_default.json
python -c "import json;d=json.load(open('$D/bench_default.json'));print(d['roofline']['frac'], d['roofline']['traffic'], d['parity_sample'])"
