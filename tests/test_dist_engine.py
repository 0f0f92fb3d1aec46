"""World-size-2 runs of the ENGINE: two processes share GPU 0
(MQ_DEVICE pins both; RCCL refuses two ranks on one GPU, so the process group is gloo), each
builds the replicated index, matches its own publish batch (the bench's per-rank seeds) on the
GPU through the C-ABI, and the all-gathered per-topic digests must equal the oracle's over both
batches. This is the harness bench.py runs under torch.distributed.run (mqmatch/dist.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _replicated_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MQ_DEVICE="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MQ_DIST_BACKEND="gloo")
    from mqmatch import dist as D
    from mqmatch import engine as E
    from mqmatch import workload as W
    from digest import engine_digests
    backend = D.init(rank)
    w = W.gen_subscriptions(60000, 6000, seed=5)
    eng = E.Engine(device=D.device_for(rank))
    eng.subscribe_bulk(w)
    tb, to = W.gen_topics(w, 3000, seed=D.topic_seed(rank))
    dg, _ = engine_digests(eng.match_batch_spans(tb, to))
    allg = D.gather_u64(dg, backend)
    D.barrier(backend)
    if rank == 0:
        out.put(np.concatenate(allg).tolist())
    D.finalize(backend)


def test_two_rank_engine_replicated(gpu_available):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replicated_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
    from mqmatch import dist as D
    from mqmatch import workload as W
    import oracle as O
    w = W.gen_subscriptions(60000, 6000, seed=5)
    orc = O.OracleIndex()
    orc.subscribe_bulk(w)
    ref = []
    for r in range(2):
        tb, to = W.gen_topics(w, 3000, seed=D.topic_seed(r))
        ref.append(orc.digest_batch(tb, to, nthreads=8)[0])
    assert got == np.concatenate(ref).tolist()
