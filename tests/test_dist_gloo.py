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
