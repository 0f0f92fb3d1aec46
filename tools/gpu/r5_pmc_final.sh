# Round 5 evidence: rocprofv3 kernel trace of the default bench step, FETCH_SIZE / WRITE_SIZE /
# TCC hit-miss passes of its kernels (walk, k_set, dedup, finish), then FETCH_SIZE / WRITE_SIZE of
# the Messages step at 100M retained (config 5) — one counter group per run
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/final
mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu"
K="k_walkf|k_set|k_dedup|k_finish|k_merge|k_walk"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py $ARGS > $O/trace.json 2> $O/trace.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $O/fetch -o run -- python3 $R/bench.py $ARGS > $O/fetch.json 2> $O/fetch.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $O/write -o run -- python3 $R/bench.py $ARGS > $O/write.json 2> $O/write.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" --output-format csv -d $O/hit -o run -- python3 $R/bench.py $ARGS > $O/hit.json 2> $O/hit.err || exit 1
MARGS="--retained 100000000 --sys 1000 --filters 100000 --steps 2 --warmup 1 --no-cpu"
MK="k_msgq|k_msg_copy"
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$MK" --output-format csv -d $O/mfetch -o run -- python3 $R/bench_messages.py $MARGS > $O/mfetch.json 2> $O/mfetch.err || exit 1
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$MK" --output-format csv -d $O/mwrite -o run -- python3 $R/bench_messages.py $MARGS > $O/mwrite.json 2> $O/mwrite.err || exit 1
