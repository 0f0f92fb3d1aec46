# Round 2: kernel trace (csv) + PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the default
# 10M span-format bench step, then the Messages bench at 10M retained (level-order image).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r2b_pmc}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_walk|k_merge|k_desc|k_scan"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py $ARGS > $D/trace.json 2> $D/trace.err || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- python3 $R/bench.py $ARGS > $D/fetch.json 2> $D/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/write -o run -- python3 $R/bench.py $ARGS > $D/write.json 2> $D/write.err || { echo "write rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/trace > $D/kernel_stats.json
python profiles/summarize.py $D/fetch $D/write --pmc > $D/pmc.json
cat $D/kernel_stats.json | head -40; cat $D/pmc.json | grep -A4 hbm_bytes
timeout -k 10 500 python -u bench_messages.py --retained 10000000 > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -5 $D/msg_10m.err; exit 1; }
cat $D/msg_10m.json
