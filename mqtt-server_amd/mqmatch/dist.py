"""Multi-process plumbing for the engine: one process per GPU.

Two modes:
  - replicated: publish topics are independent units, so the batch is partitioned across ranks
    and every rank holds a full replica of the index: no data-path collective; the process
    group carries only the timing barrier, the max-over-ranks elapsed time and test checksums;
  - sharded (north star, §8e(ii)): subscriptions are sharded by filter hash, every rank matches
    the full batch, and the ranks all-gather each topic's cross-shard nodes (exchange_xlists,
    RCCL all-gather over xGMI) so that every shard resolves its client merges exactly.

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


def _device_view(ptr, nbytes):
    """A torch uint8 CUDA tensor over engine-owned device memory (__cuda_array_interface__)."""
    import torch

    class _Buf:
        __cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (int(ptr or 0), False),
                                    "version": 3, "strides": None}
    return torch.as_tensor(_Buf(), device="cuda")


def exchange_exact(counts, ents):
    """The exchange of exchange_xlists on tensors of the process group's device: every rank's
    per-topic counts (int32, n each: all-gathered) and its entry bytes (uint8, 16 B per entry,
    any size: sent to every other rank with grouped point-to-point ops of exactly that size).
    Returns (all counts [world * n], {rank: its entry bytes} of the other ranks, entries per rank,
    the send buffer — keep it alive until the receivers are done)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    on = counts.device
    ne = torch.tensor([ents.numel() // 16], dtype=torch.int64, device=on)
    ne_all = torch.empty(world, dtype=torch.int64, device=on)
    dist.all_gather_into_tensor(ne_all, ne)
    c_all = torch.empty(world * counts.numel(), dtype=torch.int32, device=on)
    if on.type == "cuda":
        # the receive sizes come back through pinned memory while the counts' all-gather runs
        ne_pin = torch.empty(world, dtype=torch.int64, pin_memory=True)
        ne_pin.copy_(ne_all, non_blocking=True)
        sized = torch.cuda.Event()
        sized.record()
        counts_done = dist.all_gather_into_tensor(c_all, counts, async_op=True)
        sized.synchronize()
        ne_host = ne_pin.tolist()
    else:
        dist.all_gather_into_tensor(c_all, counts)
        counts_done = None
        ne_host = ne_all.tolist()
    recv = {r: torch.empty(16 * ne_host[r], dtype=torch.uint8, device=on) for r in range(world) if r != rank}
    ops = []
    for r in range(world):
        if r == rank:
            continue
        if ne_host[rank]:
            ops.append(dist.P2POp(dist.isend, ents, r))
        if ne_host[r]:
            ops.append(dist.P2POp(dist.irecv, recv[r], r))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if counts_done is not None:
        counts_done.wait()
    return c_all, recv, ne_host, ents


def exchange_xlists(x, backend):
    """Exchange every rank's exported list (mq_xlist from Engine.match_spans_begin): returns the
    other ranks' lists as XList structs over device tensors, and the tensors (keep them alive
    until mq_match_spans_end). Counts first, then exact sizes: one all-gather of the per-topic
    counts (n x 4 B per rank) and of the entry totals, then the entries themselves moved with
    grouped point-to-point sends and receives of exactly each rank's size (batch_isend_irecv:
    ncclSend / ncclRecv in one group over xGMI, SURVEY.md §5 — RCCL has no all-gather-v, and
    padding every rank to the largest one moved the largest rank's volume from every rank).
    gloo: the same through host memory."""
    import torch
    import torch.distributed as dist
    from .engine import XList
    world, rank = dist.get_world_size(), dist.get_rank()
    n = int(x.n_topics)
    dev = torch.device("cuda", torch.cuda.current_device())
    on = dev if backend == "nccl" else torch.device("cpu")
    counts = _device_view(x.counts, 4 * n).view(torch.int32) if n else torch.zeros(0, dtype=torch.int32, device=dev)
    ents = _device_view(x.ents, 16 * int(x.n_ents)) if x.n_ents else torch.zeros(0, dtype=torch.uint8, device=dev)
    c_all, recv, ne_host, mine = exchange_exact(counts.to(on), ents.to(on))
    if on.type != "cuda":
        c_all = c_all.to(dev)
        recv = {r: t.to(dev) for r, t in recv.items()}
    out = []
    for r in range(world):
        if r == rank:
            continue
        out.append(XList(n, r, c_all[r * n:].data_ptr() if n else None,
                         recv[r].data_ptr() if ne_host[r] else None, ne_host[r]))
    return out, (c_all, recv, mine)


def finalize(backend):
    if backend:
        import torch.distributed as dist
        dist.destroy_process_group()
