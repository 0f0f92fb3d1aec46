set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
for a in 0 1 2 4 7; do
  MQ_EMIT_ABLATE=$a timeout -k 10 200 python bench.py --subs 1000000 --steps 3 --warmup 1 --no-cpu > gpurun_out/abl/a$a.json 2> gpurun_out/abl/a$a.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --subs 1000000 --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --subs 1000000 --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --subs 1000000 --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --subs 1000000 --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc4.log 2>&1 || exit 1
