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
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex "k_set|k_walkf" --output-format csv -d $O/sq1 -o run -- python3 $R/bench.py $ARGS > $O/sq1.json 2> $O/sq1.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "k_set|k_walkf" --output-format csv -d $O/sq2 -o run -- python3 $R/bench.py $ARGS > $O/sq2.json 2> $O/sq2.err || exit 1
