# rocprofv3 kernel trace + PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the default 10M
# span step on the final tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r2c_prof}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_walk|k_merge|k_desc|k_scan|k_dedup|k_finish"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py $ARGS > $D/trace.json 2> $D/trace.err || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- python3 $R/bench.py $ARGS > $D/fetch.json 2> $D/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/write -o run -- python3 $R/bench.py $ARGS > $D/write.json 2> $D/write.err || { echo "write rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/trace > $D/kernel_stats.json
python profiles/summarize.py $D/fetch $D/write --pmc > $D/pmc.json
head -c 900 $D/kernel_stats.json
