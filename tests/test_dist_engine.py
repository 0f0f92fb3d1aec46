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


def _guarded(fn, rank, world, port, out):
    """A worker that fails reports its traceback through the queue (the test fails at once
    instead of waiting for a result that never comes)."""
    try:
        fn(rank, world, port, out)
    except BaseException:
        import traceback
        out.put(("error", rank, traceback.format_exc()))
        raise


def _get(q, timeout=150):
    got = q.get(timeout=timeout)
    if isinstance(got, tuple) and got and got[0] == "error":
        raise AssertionError(f"rank {got[1]} failed:\n{got[2]}")
    return got


def _replicated_worker_body(rank, world, port, out):
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


def _replicated_worker(rank, world, port, out):
    _guarded(_replicated_worker_body, rank, world, port, out)


def test_two_rank_engine_replicated(gpu_available):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replicated_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = _get(q)
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


def _sharded_worker_body(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MQ_DEVICE="0",
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MQ_DIST_BACKEND="gloo")
    import torch
    from mqmatch import dist as D
    from mqmatch import engine as E
    from mqmatch import workload as W
    from digest import engine_digest_parts
    backend = D.init(rank)
    w = W.gen_subscriptions(60000, 3000, seed=7)
    eng = E.Engine(device=D.device_for(rank), shard=rank, n_shards=world)
    eng.subscribe_bulk(w)
    tb, to = W.gen_topics(w, 3000, seed=8)  # every shard matches the same full batch
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    x = eng.match_spans_begin(d_tb.data_ptr(), d_to.data_ptr(), n)
    foreign, keep = D.exchange_xlists(x, backend)
    res = eng.match_spans_end_expanded(foreign, n)
    c, s = engine_digest_parts(res)
    parts = D.gather_u64(np.concatenate([c.astype(np.uint64).ravel(), s.ravel()]), backend)
    D.barrier(backend)
    if rank == 0:
        out.put([p.tolist() for p in parts])
    D.finalize(backend)


def _sharded_worker(rank, world, port, out):
    _guarded(_sharded_worker_body, rank, world, port, out)


def test_two_rank_engine_sharded(gpu_available):
    """The sharded mode across processes: each rank holds one shard, matches the full batch and
    exchanges its cross-shard list through the process group (gloo here; RCCL under the bench)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = _get(q)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
    from mqmatch import workload as W
    from digest import fold_parts
    import oracle as O
    n = 3000
    counts = np.zeros((n, 4), np.uint64)
    sums = np.zeros((n, 4), np.uint64)
    with np.errstate(over="ignore"):
        for p in parts:
            p = np.array(p, np.uint64)
            counts += p[:4 * n].reshape(n, 4)
            sums += p[4 * n:].reshape(n, 4)
    w = W.gen_subscriptions(60000, 3000, seed=7)
    orc = O.OracleIndex()
    orc.subscribe_bulk(w)
    tb, to = W.gen_topics(w, n, seed=8)
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=8)
    assert (counts.astype(np.int64) == ocnt).all()
    assert (fold_parts(counts, sums) == od).all()
