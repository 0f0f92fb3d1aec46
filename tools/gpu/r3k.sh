# Round 3 (session 2): the batching stage with packed submission queues (closed and open loop),
# the merge-set work distribution, PMC passes of the step's kernels, Messages at 10M retained,
# and the update path with a match step before and after each churn round.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3k}
mkdir -p $D
timeout -k 5 150 ./mqtt-server_amd/build/test_topics_index > $D/cpp.log 2>&1 || { echo "cpp rc=$?"; tail -20 $D/cpp.log; exit 1; }
tail -3 $D/cpp.log
timeout -k 10 300 mqtt-server_amd/build/latency 10000000 3 > $D/latency_10m.jsonl 2> $D/latency_10m.err || { echo "latency rc=$?"; tail -5 $D/latency_10m.err; exit 1; }
cut -c1-420 $D/latency_10m.jsonl
timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 1 --configs "9=8" --work > $D/work_10m.jsonl 2> $D/work_10m.err || { echo "work rc=$?"; tail -5 $D/work_10m.err; exit 1; }
cut -c1-1200 $D/work_10m.jsonl
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_walk|k_merge|k_desc|k_dedup|k_finish"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- python3 $R/bench.py $ARGS > $D/fetch.json 2> $D/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/write -o run -- python3 $R/bench.py $ARGS > $D/write.json 2> $D/write.err || { echo "write rc=$?"; exit 1; }
cd $R
python profiles/summarize.py $D/fetch $D/write --pmc > $D/pmc.json
grep -B2 -A6 hbm_bytes $D/pmc.json | head -80
timeout -k 10 400 python -u bench_messages.py --retained 10000000 > $D/msg_10m.json 2> $D/msg_10m.err || { echo "msg rc=$?"; tail -5 $D/msg_10m.err; exit 1; }
cut -c1-1500 $D/msg_10m.json
timeout -k 10 400 python -u tools/bench_update.py --subs 10000000 --churn 1000,10000,100000 --per-entry-sample 200000 > $D/update_10m.json 2> $D/update_10m.err || { echo "update rc=$?"; tail -5 $D/update_10m.err; exit 1; }
cut -c1-2500 $D/update_10m.json
