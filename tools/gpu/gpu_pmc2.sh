# Instruction-mix counters of k_merge / k_copy / k_walk (isolated kernels: MQ_SERIAL), 1M subs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/pmc2
mkdir -p $D
export MQ_SERIAL=1
ARGS="--subs 1000000 --steps 1 --warmup 1 --no-cpu"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "k_copy|k_walk|k_merge|k_desc" --output-format csv -d $D/a -o run -- python3 $R/bench.py $ARGS > $D/a.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_SMEM --kernel-include-regex "k_copy|k_walk|k_merge|k_desc" --output-format csv -d $D/b -o run -- python3 $R/bench.py $ARGS > $D/b.log 2>&1 || exit 1
