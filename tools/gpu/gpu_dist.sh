# Rehearsal of the multi-GPU bench path on the 1-GPU box: 2 ranks launched exactly as the driver
# does (torch.distributed.run), both pinned to GPU 0 (MQ_DEVICE) with gloo for the timing
# collectives (RCCL refuses two ranks on one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/dist
mkdir -p $D
MQ_DEVICE=0 MQ_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --subs 1000000 --steps 3 --warmup 1 \
  > $D/bench_2r.json 2> $D/bench_2r.err || exit 1
