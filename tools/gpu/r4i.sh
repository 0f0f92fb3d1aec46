# Round 4: the set pass's fold (records folded over their visits, no partner links):
# parity (set pass variants, device digests, merge-heavy cases, shards), then an A/B against
# the link path (MQ_OPT_SET_EXP bit 7) on the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4i}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -x -q --timeout 170 --timeout-method thread -k "trials or set_pass or digest_parity or many_merging or partner_map or long_lists or random_small or incremental or shard or survives" > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for v in fold links; do
  if [ $v = links ]; then export MQ_ENGINE_OPTIONS=18=128; else unset MQ_ENGINE_OPTIONS; fi
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 > $D/bench_$v.json 2> $D/bench_$v.err || { echo "bench $v rc=$?"; tail -5 $D/bench_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/bench_$v.json'))
print('$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, 'parity', (d.get('parity_sample') or {}).get('bit_exact'))
"
done
