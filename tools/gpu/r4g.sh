# Round 4: one record per gathered particle (NodeLists with the pair header, inline side array):
# smoke, the parity/shard/select suites, the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4g}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_select.py -x -q --timeout 170 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 600 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('$D/bench_default.json'))
print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, 'frac', round(d['roofline']['frac'],3), 'parity', d['parity_sample']['bit_exact'], 'e2e', round(d['end_to_end']['value']/1e6,1))
"
