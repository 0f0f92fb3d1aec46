# Round 5: SQ counters of the merge set pass and the walk (is the set pass issue- or latency-bound?)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/pmcset2
mkdir -p $O
ARGS="--variants 18=0 --rounds 1 --steps 2 --check 0"
K="k_set|k_walkf"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex "$K" --output-format csv -d $O/p1 -o run -- python3 $R/tools/ab_options.py $ARGS > $O/p1.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "$K" --output-format csv -d $O/p2 -o run -- python3 $R/tools/ab_options.py $ARGS > $O/p2.log 2>&1 || exit 1
