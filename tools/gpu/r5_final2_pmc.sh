# Round 5 final PMC: FETCH_SIZE / WRITE_SIZE / TCC hit-miss of the default step's kernels (one
# counter group per run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/final2pmc
mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu"
K="k_walkf|k_set|k_dedup|k_finish|k_merge|k_walk"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $O/fetch -o run -- python3 $R/bench.py $ARGS > $O/fetch.json 2> $O/fetch.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $O/write -o run -- python3 $R/bench.py $ARGS > $O/write.json 2> $O/write.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" --output-format csv -d $O/hit -o run -- python3 $R/bench.py $ARGS > $O/hit.json 2> $O/hit.err || exit 1
