"""Device-side SelectShared (k_pick; SURVEY.md §8f.3, topics.go:320-333).

Go keeps the first member of each Shared[filter] map in random iteration order, so any member
is a conformant pick; the engine picks the member with the smallest client id. Checked against
the engine's own full Shared rows (themselves bit-exact against the oracle in
test_gpu_parity.py) and, on a small case, against the oracle's Shared maps directly.
"""
import random

import numpy as np
import pytest

import oracle as O
from adapters import OracleAdapter

pytestmark = pytest.mark.gpu


def _expected_picks(res, t):
    b, n = int(res["shared_base"][t]), int(res["n_shared"][t])
    best = {}
    for f, c in res["shared"][b:b + n]:
        f, c = int(f), int(c)
        if f not in best or c < best[f]:
            best[f] = c
    return best


def _picks(res, t):
    b, n = int(res["shared_base"][t]), int(res["n_shared"][t])
    rows = [(int(f), int(c)) for f, c in res["shared"][b:b + n]]
    d = dict(rows)
    assert len(d) == len(rows), "two picks for one filter"
    return d


def _pair(w):
    from mqmatch import engine as E
    full, sel = E.Engine(), E.Engine(select_shared=True)
    assert (full.subscribe_bulk(w) == sel.subscribe_bulk(w)).all()
    return full, sel


def _check_batch(full, sel, tb, to, fmt="rows"):
    a = full.match_batch(tb, to)
    b = sel.match_batch_spans(tb, to) if fmt == "spans" else sel.match_batch(tb, to)
    for k in ("sub_base", "sub_cap", "n_client", "n_ident", "n_inline") + (("shared_base",) if fmt == "rows" else ()):
        assert (a[k] == b[k]).all(), k
    assert (a["rows"] == b["rows"]).all() and (a["inline"] == b["inline"]).all()
    n_picked = 0
    for t in range(len(to) - 1):
        assert _picks(b, t) == _expected_picks(a, t), t
        n_picked += int(b["n_shared"][t])
    return a, b, n_picked


@pytest.mark.parametrize("fmt", ["rows", "spans"])
def test_select_shared_workload(fmt, gpu_available):
    from mqmatch import workload as W
    w = W.gen_subscriptions(60000, 3000, seed=71)
    full, sel = _pair(w)
    tb, to = W.gen_topics(w, 8000, seed=72)
    a, b, n_picked = _check_batch(full, sel, tb, to, fmt)
    assert n_picked > 0 and n_picked < int(a["n_shared"].sum())


@pytest.mark.parametrize("fmt", ["rows", "spans"])
def test_select_shared_many_filters_per_topic(fmt, gpu_available):
    """More distinct shared filters in one topic than k_pick's LDS table holds: the topic is
    re-run in hash partitions."""
    from mqmatch import engine as E
    full, sel = E.Engine(), E.Engine(select_shared=True)
    r = random.Random(73)
    fid = 0
    for g in range(3000):
        for f in (f"$share/g{g}/a/b", f"$SHARE/h{g}/a/+", f"$share/k{g}/#"):
            for _ in range(r.randint(1, 4)):
                c = r.randrange(100000)
                for e in (full, sel):
                    e.subscribe(f, c, fid, qos=1)
            fid += 1
    for e in (full, sel):
        e.subscribe("a/b", 5, fid, qos=2)
    topics = ["a/b", "a/c", "x", "a", "a/b/c", "$SYS/a"]
    tb, to = E.pack_strings(topics)
    a, b, n_picked = _check_batch(full, sel, tb, to, fmt)
    assert int(b["n_shared"][0]) == 9000 and n_picked == 9000 + 6000 + 3000 * 4


def test_select_shared_vs_oracle_and_server_flow(gpu_available):
    """The picked member is one of the oracle's Shared[filter] members (the smallest client id),
    and the broker flow (SelectShared + MergeSharedSelected, server.go:1001-1007) over the
    device picks gives the Go result for that pick."""
    from mqmatch import engine as E
    r = random.Random(74)
    ti, o = E.TopicsIndex(0, select_shared=True), OracleAdapter()
    segs = ["a", "b", "+", "#", "c"]
    for _ in range(400):
        f = "/".join(r.choice(segs) for _ in range(r.randint(1, 3)))
        if r.random() < 0.6:
            f = f"{r.choice(['$share', '$SHARE'])}/g{r.randrange(4)}/{f}"
        c = f"c{r.randrange(30)}"
        s = E.Subscription(f, r.choice([0, 0, 5, 7]), r.randint(0, 2), r.random() < 0.2)
        ti.subscribe(c, s)
        o.subscribe(c, f, qos=s.qos, identifier=s.identifier, no_local=s.no_local)
    topics = ["a", "a/b", "a/b/c", "b/c", "c", "a/c/b", "$SYS/a"]
    for t, got in zip(topics, ti.subscribers_batch(topics)):
        want = o.subscribers(t)
        assert set(got.shared) == set(want["shared"]), t
        for f, members in got.shared.items():
            assert len(members) == 1
            (client,) = members
            assert client in want["shared"][f]
            assert ti.client_ids[client] == min(ti.client_ids[c] for c in want["shared"][f])
        got.select_shared()
        got.merge_shared_selected()
        assert set(got.subscriptions) == set(want["subscriptions"]) | {
            next(iter(m)) for m in got.shared.values()}, t


def test_select_shared_device_api(gpu_available):
    """mq_select_shared_device on each chunk inside a chunk consumer (torch-owned output
    buffers, the chunk stream) equals the MQ_CFG_SELECT_SHARED batch results."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(50000, 5000, seed=75)
    full, sel = _pair(w)
    full.set_option(E.OPT_CHUNK_ROWS, 150000)
    tb, to = W.gen_topics(w, 20000, seed=76)
    n = len(to) - 1
    want = sel.match_batch(tb, to)
    got_n = np.zeros(n, np.uint32)
    got = {}
    keep = []

    def consume(chunk, first, stream):
        d_sel = torch.empty(max(1, chunk.n_shared_rows) * 2, dtype=torch.int32, device="cuda")
        d_n = torch.empty(max(1, chunk.n_topics), dtype=torch.int32, device="cuda")
        d_top = torch.empty(chunk.n_topics * 12, dtype=torch.int32, device="cuda")
        full.select_shared_device(chunk, stream, d_sel.data_ptr(), d_n.data_ptr())
        import ctypes as C
        hip = C.CDLL("libamdhip64.so")
        hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        assert hip.hipMemcpyAsync(d_top.data_ptr(), chunk.topics, chunk.n_topics * 48, 3, stream) == 0
        hip.hipStreamSynchronize.argtypes = [C.c_void_p]
        assert hip.hipStreamSynchronize(stream) == 0
        keep.append((first, chunk.n_topics, d_sel.cpu().numpy().view(np.uint32).reshape(-1, 2),
                     d_n.cpu().numpy().view(np.uint32)[:chunk.n_topics],
                     d_top.cpu().numpy().view(np.uint32).reshape(-1, 12)))

    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    s = torch.cuda.Stream()
    full.match_device_chunks(d_tb.data_ptr(), d_to.data_ptr(), n, s.cuda_stream, consume)
    torch.cuda.synchronize()
    assert len(keep) == full.match_chunks() > 1
    for first, nt, rows, cnt, top in keep:
        sb = top[:, 2].astype(np.uint64) | (top[:, 3].astype(np.uint64) << np.uint64(32))
        for k in range(nt):
            t = first + k
            g = {int(f): int(c) for f, c in rows[int(sb[k]):int(sb[k]) + int(cnt[k])]}
            assert len(g) == int(cnt[k])
            assert g == _picks(want, t), t
