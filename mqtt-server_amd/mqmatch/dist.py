"""Multi-process plumbing for the engine: one process per GPU.

Publish topics are independent units, so the batch is partitioned across ranks and every rank
holds a full replica of the index: no data-path collective. The process group carries only
the timing barrier, the max-over-ranks elapsed time and (in tests) result checksums.

Backend: "nccl" (RCCL over xGMI) on GPUs; `MQ_DIST_BACKEND=gloo` rehearses the same code on
CPU or with several ranks sharing one GPU (RCCL refuses duplicate GPUs in a communicator).
"""
import os

import numpy as np

from .workload import BASE_SEED


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def topic_seed(rank):
    """Each rank draws its own publish batch (weak scaling: per-GPU work is fixed)."""
    return BASE_SEED + 1000 * rank


def device_for(local_rank):
    """GPU ordinal of this rank; MQ_DEVICE pins every rank to one GPU (rehearsal)."""
    d = os.environ.get("MQ_DEVICE")
    return int(d) if d is not None else local_rank


def init(local_rank):
    """Initialise the process group when WORLD_SIZE > 1; returns the backend or None."""
    import torch
    import torch.distributed as dist
    rank, world, _ = env_rank()
    if world <= 1:
        return None
    backend = os.environ.get("MQ_DIST_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", device_for(local_rank)))
    else:
        dist.init_process_group(backend)
    return backend


def _tensor(x, backend):
    import torch
    t = torch.tensor(x, dtype=torch.float64)
    return t.cuda() if backend == "nccl" else t


def barrier(backend):
    if backend:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, backend):
    """Max of a float over ranks (the slowest rank defines whole-job time)."""
    if not backend:
        return float(x)
    import torch.distributed as dist
    t = _tensor([x], backend)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, backend):
    if not backend:
        return float(x)
    import torch.distributed as dist
    t = _tensor([x], backend)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_u64(arr, backend):
    """All-gather equal-length u64 arrays (as int64) -> list per rank."""
    if not backend:
        return [arr]
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(arr).view(np.int64))
    if backend == "nccl":
        t = t.cuda()
    outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, t)
    return [o.cpu().numpy().view(np.uint64) for o in outs]


def finalize(backend):
    if backend:
        import torch.distributed as dist
        dist.destroy_process_group()
