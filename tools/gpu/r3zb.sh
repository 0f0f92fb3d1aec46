# Round 3 (session 2): the host result's bytes per array (end_to_end), the set pass variants'
# parity, and config 4 with the merge stage priced on the topics its kernels resolve.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3zb}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "set_pass_variants or spans_format_shape or spans_device_matches_host" -x -v --timeout 170 --timeout-method thread > $D/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
cut -c1-300 $D/bench_default.json
timeout -k 10 400 python -u bench.py --mix iot --subs 50000000 --no-cpu > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -5 $D/bench_iot_50m.err; exit 1; }
cut -c1-300 $D/bench_iot_50m.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $D/e2e_trace -o run -- python3 $R/tools/e2e_probe.py > $D/e2e_probe.jsonl 2> $D/e2e_probe.err || { echo "e2e probe rc=$?"; tail -5 $D/e2e_probe.err; exit 1; }
cut -c1-400 $D/e2e_probe.jsonl
