# Round 3: counter calibration (tools/randbench: known bytes, coalesced stream and random 32 B
# loads), then the default span step under rocprofv3 (kernel trace; FETCH_SIZE, WRITE_SIZE and SQ
# passes of the frontier walk and the merge stage), then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/${1:-r3b}
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
cd $R && timeout -k 10 300 python -u tools/tune_spans.py --subs 10000000 --reps 2 --configs "9=8;9=1" > $D/tune_walk_wpe.jsonl 2> $D/tune_walk_wpe.err || { echo "tune rc=$?"; tail -5 $D/tune_walk_wpe.err; exit 1; }
cut -c1-300 $D/tune_walk_wpe.jsonl
cd /tmp
timeout -k 10 120 $R/tools/randbench > $D/randbench.txt 2>&1 || { echo "randbench rc=$?"; exit 1; }
cat $D/randbench.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/rb_fetch -o run -- $R/tools/randbench > /dev/null 2>$D/rb_fetch.err || { echo "rb fetch rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/rb_write -o run -- $R/tools/randbench > /dev/null 2>$D/rb_write.err || { echo "rb write rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $D/rb_req -o run -- $R/tools/randbench > /dev/null 2>$D/rb_req.err || { echo "rb req rc=$?"; }
ARGS="--steps 3 --warmup 1 --no-cpu"
KR="k_walk|k_merge|k_desc|k_scan|k_dedup|k_finish"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py $ARGS > $D/trace.json 2> $D/trace.err || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/fetch -o run -- python3 $R/bench.py $ARGS > $D/fetch.json 2> $D/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" --output-format csv -d $D/write -o run -- python3 $R/bench.py $ARGS > $D/write.json 2> $D/write.err || { echo "write rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "k_walk|k_merge" --output-format csv -d $D/sq -o run -- python3 $R/bench.py $ARGS > $D/sq.json 2> $D/sq.err || { echo "sq rc=$?"; }
cd $R
python profiles/summarize.py $D/trace > $D/kernel_stats.json
python profiles/summarize.py $D/fetch $D/write $D/sq --pmc > $D/pmc.json
python profiles/summarize.py $D/rb_fetch $D/rb_write $D/rb_req --pmc > $D/rb_pmc.json
timeout -k 10 600 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench rc=$?"; tail -5 $D/bench_default.err; exit 1; }
python tools/show.py $D/bench_default.json
