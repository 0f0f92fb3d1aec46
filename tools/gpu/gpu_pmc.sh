# PMC passes (one counter group per run) + kernel-trace stats of the 10M bench step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
ARGS="--steps 1 --warmup 1 --no-cpu ${BENCH_ARGS}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc/trace -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/trace.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_copy|k_walk|k_merge|k_desc" --output-format csv -d $R/gpurun_out/pmc/fetch -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_copy|k_walk|k_merge|k_desc" --output-format csv -d $R/gpurun_out/pmc/write -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/write.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_copy|k_walk|k_merge|k_desc" --output-format csv -d $R/gpurun_out/pmc/hit -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/hit.log 2>&1 || exit 1
