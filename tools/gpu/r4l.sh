# Round 4 evidence on the committed tree: the kernel trace (rocprofv3 --kernel-trace --stats) and
# PMC traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of the 10M step, the device rate at the Go
# stage's 16k batch, and config 4 (50M IoT) with its parity sample (oracle side in a child).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r4l}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_walk|k_merge|k_desc|k_dedup|k_finish|k_reset|k_readback|k_span_pack|k_set_pack|k_mrow_pack|k_host_rebase"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py $ARGS > $D/trace.json 2> $D/trace.err || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- python3 $R/bench.py $ARGS > $D/fetch.json 2> $D/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/write -o run -- python3 $R/bench.py $ARGS > $D/write.json 2> $D/write.err || { echo "write rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/trace > $D/kernel_stats.json
python profiles/summarize.py $D/fetch $D/write --pmc > $D/pmc.json
head -c 1200 $D/kernel_stats.json; echo
timeout -k 10 300 python -u bench.py --topics 16384 --steps 200 --warmup 20 --no-cpu > $D/bench_16k.json 2> $D/bench_16k.err || { echo "16k rc=$?"; tail -5 $D/bench_16k.err; exit 1; }
cut -c1-300 $D/bench_16k.json
timeout -k 10 900 python -u bench.py --mix iot --subs 50000000 --steps 10 > $D/bench_iot_50m.json 2> $D/bench_iot_50m.err || { echo "iot rc=$?"; tail -5 $D/bench_iot_50m.err; exit 1; }
cut -c1-400 $D/bench_iot_50m.json
