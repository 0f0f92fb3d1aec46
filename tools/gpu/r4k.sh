# Round 4: the default bench (fold vs partner links), Messages at 10M, the C++ mirror (update
# latency under read load), then the parity suites touched this round.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4k}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
for v in fold links; do
  if [ $v = links ]; then export MQ_ENGINE_OPTIONS=18=128; else unset MQ_ENGINE_OPTIONS; fi
  timeout -k 10 400 python -u bench.py --steps 10 > $D/bench_$v.json 2> $D/bench_$v.err || { echo "bench $v rc=$?"; tail -5 $D/bench_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/bench_$v.json'))
e=d.get('end_to_end') or {}
print('$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, 'parity', (d.get('parity_sample') or {}).get('bit_exact'), 'e2e', round(e.get('value',0)/1e6,1), 'pipelined', round((e.get('pipelined') or {}).get('value',0)/1e6,1), (e.get('pipelined') or {}).get('bytes_per_topic'))
"
done
unset MQ_ENGINE_OPTIONS
timeout -k 10 400 python -u bench_messages.py --retained 10000000 > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -5 $D/msg_10m.err; exit 1; }
python3 -c "
import json; d=json.load(open('$D/msg_10m.json'))
print('msg10m', round(d['value']/1e6,1), 'M filters/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, d.get('parity_sample'))
"
timeout -k 10 300 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1; echo "cpp rc=$?"
grep -E "slowest|over 2 ms|passed|FAIL|REQUIRE" $D/cpp.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_select.py -x -q --timeout 170 --timeout-method thread -k "not cpp_host" > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
