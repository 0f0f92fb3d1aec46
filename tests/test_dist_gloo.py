"""World-size-2 rehearsal of the multi-GPU path on CPU with gloo.

Each rank builds the same replicated index (oracle restatement here: no GPU on CPU), draws its
own publish batch with the per-rank seed, and reports per-topic digests; the all-gathered
digests must equal a single-process run over every rank's batch, and the max/sum reductions
must see both ranks. This is the exact harness bench.py uses (mqmatch/dist.py)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MQ_DIST_BACKEND="gloo")
    from mqmatch import dist as D
    from mqmatch import workload as W
    import oracle as O
    backend = D.init(rank)
    w = W.gen_subscriptions(5000, 500, seed=3)
    orc = O.OracleIndex()
    orc.subscribe_bulk(w)
    tb, to = W.gen_topics(w, 300, seed=D.topic_seed(rank))
    dg, _, _ = orc.digest_batch(tb, to, nthreads=1)
    allg = D.gather_u64(dg, backend)
    mx = D.max_over_ranks(float(rank + 1), backend)
    sm = D.sum_over_ranks(1.0, backend)
    D.barrier(backend)
    if rank == 0:
        out.put((np.concatenate(allg).tolist(), mx, sm))
    D.finalize(backend)


def test_two_rank_gloo_partition():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, mx, sm = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mx == 2.0 and sm == 2.0
    # single-process reference over both ranks' batches
    import sys
    sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
    from mqmatch import dist as D
    from mqmatch import workload as W
    import oracle as O
    w = W.gen_subscriptions(5000, 500, seed=3)
    orc = O.OracleIndex()
    orc.subscribe_bulk(w)
    ref = []
    for r in range(2):
        tb, to = W.gen_topics(w, 300, seed=D.topic_seed(r))
        ref.append(orc.digest_batch(tb, to, nthreads=1)[0])
    assert got == np.concatenate(ref).tolist()


def _xworker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MQ_DIST_BACKEND="gloo")
    import torch
    from mqmatch import dist as D
    backend = D.init(rank)
    n = 7
    # rank r exports r * 5 entries (rank 0 none): uneven sizes, one rank empty
    counts = torch.tensor([(rank * 5 * (t + 1)) // 28 - (rank * 5 * t) // 28 for t in range(n)], dtype=torch.int32)
    ents = torch.arange(16 * rank * 5, dtype=torch.int64).to(torch.uint8) + rank
    c_all, recv, ne, _ = D.exchange_exact(counts, ents)
    D.barrier(backend)
    out.put((rank, c_all.tolist(), {r: t.tolist() for r, t in recv.items()}, ne))
    D.finalize(backend)


def test_exact_size_exchange_three_ranks():
    """dist.exchange_exact (the sharded mode's cross-shard list exchange): counts all-gathered,
    entries moved with grouped point-to-point ops of exactly each rank's size (uneven, one rank
    exporting nothing)."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xworker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, c_all, recv, ne = q.get(timeout=240)
        res[rank] = (c_all, recv, ne)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 7
    want_counts = []
    for r in range(world):
        want_counts += [(r * 5 * (t + 1)) // 28 - (r * 5 * t) // 28 for t in range(n)]
    for rank, (c_all, recv, ne) in res.items():
        assert ne == [0, 5, 10]
        assert c_all == want_counts
        assert sorted(recv) == [r for r in range(world) if r != rank]
        for r, got in recv.items():
            assert got == [(i + r) % 256 for i in range(16 * r * 5)]
