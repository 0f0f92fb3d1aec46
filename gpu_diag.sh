# Diagnosis: per-topic k_merge phase cycles, isolated (MQ_SERIAL) and overlapped with k_copy.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag
D=gpurun_out/diag
MQ_SERIAL=1 MQ_COPY_BLOCKS_PER_CU=8 MQ_MERGE_STATS=$D/ts_serial_10m.bin timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu > $D/ts_serial_10m.json 2> $D/ts_serial_10m.err || exit 1
MQ_COPY_BLOCKS_PER_CU=8 MQ_MERGE_STATS=$D/ts_ovl_10m.bin timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu > $D/ts_ovl_10m.json 2> $D/ts_ovl_10m.err || exit 1
