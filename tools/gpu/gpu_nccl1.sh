# The driver's multi-GPU launch line at one rank: torch.distributed.run + RCCL ("nccl") process
# group on the 1-GPU box (N>1 needs a node with that many GPUs).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/nccl1
mkdir -p $D
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 5 --warmup 2 \
  > $D/bench_torchrun_1r.json 2> $D/bench_torchrun_1r.err || exit 1
