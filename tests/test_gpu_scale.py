"""Parity at the benchmarks' own scale: the headline configuration (10M subscriptions, config-3
mix, SURVEY.md §8d generator) unsharded and sharded 8 ways, the IoT fan-in mix, and the retained
reverse match (config 5) at 10M retained topics x 100k filters — every one digest-equal to the
oracle. The 10M workload and its oracle digests are built once for the module (the oracle is
freed before the engines are built). Besides the sample, every topic of the 1M-topic batch is
checked for size-independent properties of the span format."""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle as O
from digest import engine_digests

pytestmark = pytest.mark.gpu

NS = 4096  # topics of the bench batch checked against the oracle
NS_SHARD = 16384  # ... and by the 8-shard test
THREADS = min(16, os.cpu_count() or 8)


@pytest.fixture(scope="module")
def config3():
    """bench.py's index (10M config-3 subscriptions) and rank-0 batch (1M topics), with the
    oracle's answers for the batch's first NS topics."""
    from mqmatch import workload as W
    w = W.gen_subscriptions(10_000_000, 1_000_000, seed=W.BASE_SEED)
    tb, to = W.gen_topics(w, 1_000_000, seed=W.BASE_SEED)
    orc = O.OracleIndex()
    new = orc.subscribe_bulk(w)
    od, ocnt, _ = orc.digest_batch(tb, to[:NS_SHARD + 1], nthreads=THREADS)
    orc.close()
    del orc
    return {"w": w, "new": new, "tb": tb, "to": to, "od": od[:NS], "ocnt": ocnt[:NS], "od_s": od, "ocnt_s": ocnt}


def _check(dg, cnt, od, ocnt, what):
    bad = np.nonzero(dg != od)[0]
    assert len(bad) == 0, f"{what}: {len(bad)} of {len(dg)} topics differ, first {bad[:5]}"
    assert (cnt == ocnt).all(), what


@pytest.mark.timeout(900)
def test_headline_10m_subscriptions(config3, gpu_available):
    """The headline index through every result path: host spans and rows on the sample, and the
    timed path itself — one-sync mq_match_spans_device on the whole 1M-topic batch (the walk
    trials, then the walk they chose), the frontier walk with k_desc fused forced, and the walk
    thread per topic forced — each device result's first NS topics expanded as a device consumer
    would and compared with the oracle."""
    import torch
    from mqmatch import engine as E
    c = config3
    tb, to, od, ocnt = c["tb"], c["to"], c["od"], c["ocnt"]
    eng = E.Engine(expected_subs=10_000_000)
    assert (eng.subscribe_bulk(c["w"]) == c["new"]).all()
    for fmt, res in (("host spans", eng.match_batch_spans(tb, to[:NS + 1])), ("rows", eng.match_batch(tb, to[:NS + 1]))):
        dg, cnt = engine_digests(res)
        _check(dg, cnt, od, ocnt, fmt)
    assert ocnt[:, 0].mean() > 1000  # the workload really fans out
    # the timed path: device results of the whole batch (>= 64k topics: trials, merge-set dedup
    # over the batch, one host synchronisation)
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    torch.cuda.synchronize()
    runs = [(f"trial {k + 1}", None) for k in range(6)] + [("chosen walk", None),
            ("frontier walk + fused desc", 16), ("walk thread per topic", 0)]
    for what, group in runs:
        if group is not None:
            eng.set_option(E.OPT_WALK_GROUP, group)
        eng.profile(True)
        eng.profile_reset()
        r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
        prof = eng.profile_read()
        eng.profile(False)
        res = E.expand_device_spans(r, n, NS)
        dg, cnt = engine_digests(res)
        _check(dg, cnt, od, ocnt, f"device spans, {what}")
        assert res["set_topics"] > NS // 2, what  # the merge-set dedup path answered most topics
        assert "walk" in prof, prof
    del d_tb, d_to
    # every topic of the full batch: span-format invariants, independent of the oracle
    a = eng.match_spans(tb, to)
    t = a["topics"]
    assert (t["n_client"] <= t["n_rows"]).all() and (t["n_ident"] <= t["n_rows"] - t["n_client"]).all()
    # patch ranges are reserved per topic before resolving (hit-list records); the written part
    # of each range is n_patches; topics of a merge set name its patches (packed, ABI v7)
    setf = (t["flags"] & 1) != 0
    assert int(t["n_spans"].sum()) == len(a["spans"]) and int(t["n_patches"][~setf].sum()) <= len(a["patches"])
    tid, prow, _ = E.host_topic_patches(a)
    assert len(tid) == int(t["n_patches"].sum()) and (prow < t["n_rows"][tid]).all()
    sb, ns = t["span_base"].astype(np.int64), t["n_spans"].astype(np.int64)
    cs = np.concatenate(([0], np.cumsum(a["spans"][:, 1].astype(np.int64))))
    assert (cs[sb + ns] - cs[sb] == t["n_rows"]).all()  # spans cover exactly the gathered records
    cs = np.concatenate(([0], np.cumsum(a["spans"][:, 3].astype(np.int64))))
    assert (cs[sb + ns] - cs[sb] == t["n_shared"]).all()
    # a patch changes a row; a topic whose records all belong to distinct clients needs none but
    # merge-base Qos/NoLocal rewrites, which exist only where n_client < n_rows
    no_merge = t["n_client"] == t["n_rows"]
    assert (t["n_patches"][no_merge] == 0).all()
    assert int((t["n_rows"] - t["n_client"]).sum()) <= int(t["n_patches"].sum())
    del a
    eng.close()


@pytest.mark.timeout(900)
def test_config3_eight_shards_10m(config3, gpu_available):
    """Config 3 in its stated form: the 10M config-3 subscriptions sharded by filter hash over 8
    shard handles (one GPU here), every shard matching the full NS_SHARD-topic batch, the exported
    cross-shard lists exchanged, each shard resolving its own records; the shards' disjoint
    device results add up to the oracle's digests, bit for bit (host results too)."""
    from mqmatch import engine as E
    from test_gpu_shard import _sharded_digests
    c = config3
    tb, to = c["tb"], c["to"][:NS_SHARD + 1].copy()
    shards = [E.Engine(shard=k, n_shards=8, expected_subs=10_000_000 // 8) for k in range(8)]
    # the shards build in parallel (the bulk build releases the GIL): each applies every entry
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda e: e.subscribe_bulk(c["w"]), shards))
    new = c["new"]
    for g in got:
        assert (g <= new).all()
    assert (np.bitwise_or.reduce(np.stack(got), axis=0) == new).all()  # the owner answers
    for device in (True, False):
        dg, cnt, n_ents = _sharded_digests(shards, tb, to, device=device)
        _check(dg, cnt, c["od_s"], c["ocnt_s"], f"8 shards, {'device' if device else 'host'} results")
        assert n_ents > 0
    for e in shards:
        e.close()


def test_iot_5m_subscriptions(gpu_available):
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(5_000_000, 5_000_000, seed=W.BASE_SEED, mix=W.MIX_IOT)
    eng = E.Engine(expected_subs=5_000_000)
    new = eng.subscribe_bulk(w)
    orc = O.OracleIndex()
    assert (orc.subscribe_bulk(w) == new).all()
    tb, to = W.gen_topics(w, 20000, seed=W.BASE_SEED, mix=W.MIX_IOT)
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=THREADS)
    for fmt in ("spans", "rows"):
        res = eng.match_batch_spans(tb, to) if fmt == "spans" else eng.match_batch(tb, to)
        dg, cnt = engine_digests(res)
        _check(dg, cnt, od, ocnt, fmt)


@pytest.mark.timeout(900)
def test_iot_5m_half_load_edge_table(gpu_available):
    """Config 4's probe regime at a tenth of its size: the 50M IoT index is held at an edge table
    of 2^30 slots at most half full (mqmatch.h MQ_OPT_EDGE_LOAD), where probe chains are longest;
    here the 5M IoT index is forced to the same bound (MQ_OPT_EDGE_LOAD 2). The timed path —
    one-sync mq_match_spans_device over a 256k-topic batch: the walk trials, then each walk
    forced — and host spans, the first 20k topics digest-equal to the oracle (topics.go:593-648)."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    ns = 20000
    w = W.gen_subscriptions(5_000_000, 5_000_000, seed=W.BASE_SEED + 40, mix=W.MIX_IOT)
    eng = E.Engine(expected_subs=5_000_000)
    eng.set_option(E.OPT_EDGE_LOAD, 2)
    new = eng.subscribe_bulk(w)
    st = eng.stats()
    assert st["edge_load"] == 2 and st["edges"] * 4 >= st["edge_capacity"], st  # 1/4 .. 1/2 full
    tb, to = W.gen_topics(w, 1 << 18, seed=W.BASE_SEED + 41, mix=W.MIX_IOT)
    orc = O.OracleIndex()
    assert (orc.subscribe_bulk(w) == new).all()
    od, ocnt, _ = orc.digest_batch(tb, to[:ns + 1], nthreads=THREADS)
    orc.close()
    del orc
    dg, cnt = engine_digests(eng.match_batch_spans(tb, to[:ns + 1]))
    _check(dg, cnt, od, ocnt, "host spans")
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    torch.cuda.synchronize()
    runs = [(f"trial {k + 1}", None) for k in range(6)] + [("chosen walk", None),
            ("frontier walk + fused desc", 16), ("walk thread per topic", 0)]
    for what, group in runs:
        if group is not None:
            eng.set_option(E.OPT_WALK_GROUP, group)
        r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
        dg, cnt = engine_digests(E.expand_device_spans(r, n, ns))
        _check(dg, cnt, od, ocnt, f"device spans, {what}")
    del d_tb, d_to
    eng.close()


@pytest.mark.timeout(900)
def test_messages_10m_retained_100k_filters(gpu_available):
    """Config 5 at a tenth of its size (bench_messages.py's default workload and seeds): 10M
    retained topics (1k $SYS) x 100k wildcard filters through mq_messages_device, every filter's
    handle set digest-equal to the fast restatement (FastMsgIndex, itself digest-checked against
    the oracle here on the first 4096 filters)."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    rb, ro, hd, rh = W.gen_retained(10_000_000, n_sys=1000, seed=W.BASE_SEED + 3)
    fb, fo = W.gen_msg_filters(rh, 100_000, seed=W.BASE_SEED + 4)
    del rh
    n = len(fo) - 1
    orc = O.OracleIndex()
    orc.retain_bulk(rb, ro, hd)
    fast = orc.fast_messages()
    fd, fcnt = fast.digest_batch(fb, fo, nthreads=THREADS)
    od, ocnt, _ = orc.messages_digest_batch(fb, fo[:4097], nthreads=THREADS)
    assert (fd[:4096] == od).all() and (fcnt[:4096] == ocnt).all()
    fast.close()
    orc.close()
    del fast, orc
    eng = E.Engine()
    eng.retain_bulk(rb, ro, hd)
    d_fb = torch.from_numpy(np.concatenate([fb, np.zeros(16, np.uint8)])).cuda()
    d_fo = torch.from_numpy(fo.view(np.int64)).cuda()
    torch.cuda.synchronize()
    r = eng.messages_device(d_fb.data_ptr(), d_fo.data_ptr(), n, None)
    base, count, hs = E.device_messages(r, n)
    assert (count == fcnt).all()
    dg = O.handle_digests(base, count, hs, nthreads=THREADS)
    bad = np.nonzero(dg != fd)[0]
    assert len(bad) == 0, f"{len(bad)} of {n} filters differ, first {bad[:5]}"
    assert int(count.sum()) > 10 * n  # the filters fan out
    del hs
    # the same batch as runs at the boundary (mq_messages_runs_device: bench_messages.py's step)
    res = E.device_messages_runs(eng.messages_runs_device(d_fb.data_ptr(), d_fo.data_ptr(), n, None), n)
    assert (res["count"] == fcnt).all()
    bad = np.nonzero(O.run_digests(res, nthreads=THREADS) != fd)[0]
    assert len(bad) == 0, f"runs: {len(bad)} of {n} filters differ, first {bad[:5]}"
    assert len(res["runs"]) * 8 < int(fcnt.sum())
    eng.close()
