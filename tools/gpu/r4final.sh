# Round 4 final evidence: smoke, the default bench line, the C++ mirror, the kernel trace, PMC traffic
# (FETCH_SIZE, WRITE_SIZE) and the L2 hit / miss counts of the walk and merge kernels (TCC_HIT, TCC_MISS).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4final}
mkdir -p $D
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('$D/bench_default.json'))
e=d.get('end_to_end') or {}
print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, 'parity', (d.get('parity_sample') or {}).get('bit_exact'), 'e2e', round(e.get('value',0)/1e6,1), 'pipelined', round((e.get('pipelined') or {}).get('value',0)/1e6,1), (e.get('pipelined') or {}).get('runs_ms'))
"
cat /sys/fs/cgroup/cpu.stat > $D/cpu_stat_before.txt 2>/dev/null; cat /sys/fs/cgroup/cpu.max > $D/cpu_max.txt 2>/dev/null
timeout -k 10 300 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1; echo "cpp rc=$?"
cat /sys/fs/cgroup/cpu.stat > $D/cpu_stat_after.txt 2>/dev/null
grep -E "slowest|over 2 ms|passed|FAIL|REQUIRE" $D/cpp.log
echo "cpu.max: $(cat $D/cpu_max.txt 2>/dev/null)"; paste $D/cpu_stat_before.txt $D/cpu_stat_after.txt 2>/dev/null | head -8
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_walk|k_merge|k_desc|k_dedup|k_finish|k_reset|k_readback"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py $ARGS > $D/trace.json 2> $D/trace.err || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- python3 $R/bench.py $ARGS > $D/fetch.json 2> $D/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/write -o run -- python3 $R/bench.py $ARGS > $D/write.json 2> $D/write.err || { echo "write rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$KR" --output-format csv -d $D/tcc -o run -- python3 $R/bench.py $ARGS > $D/tcc.json 2> $D/tcc.err || { echo "tcc rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/tcc --pmc > $D/tcc_summary.json || true
python profiles/summarize.py $D/trace > $D/kernel_stats.json
python profiles/summarize.py $D/fetch $D/write --pmc > $D/pmc.json
head -c 1500 $D/kernel_stats.json; echo
