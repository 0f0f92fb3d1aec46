"""Parity of the HIP path (through the C-ABI) with the oracle, bit-exact on ids.

Small cases compare the rematerialised Go-shaped Subscribers maps topic by topic; workload-scale
cases compare per-topic canonical digests of every row (tests/digest.py). Edge cases follow the
reference's tests and quirk register: empty topics, '$' topics, empty
levels, literal '+'/'#' topic levels, long (hashed) segments, deep topics, Unicode $share,
inline last-write, incremental updates between batches, chunked outputs.
"""
import functools
import os
import random

import numpy as np
import pytest

from adapters import EngineAdapter, OracleAdapter, canonical
from digest import engine_digests
from kat_cases import KATS, MESSAGE_KATS
import oracle as O

pytestmark = pytest.mark.gpu


FORMATS = ["spans", "rows"]  # mq_match_spans (+ mq_spans_expand) and mq_match_batch


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("kat", KATS + MESSAGE_KATS, ids=lambda f: f.__name__)
def test_engine_kat(kat, fmt, gpu_available):
    kat(functools.partial(EngineAdapter, fmt))


SEGS = ["a", "b", "c", "", "+", "#", "$SYS", "$share", "$SHARE", "$ſhare", "g", "sport",
        "averyveryverylongsegment", "averyveryverylongsegmenz", "x", "ü"]
TSEGS = ["a", "b", "c", "", "$SYS", "$share", "g", "sport", "averyveryverylongsegment",
         "averyveryverylongsegmenz", "x", "ü", "$x"]


def rand_filter(r, segs=SEGS):
    return "/".join(r.choice(segs) for _ in range(r.randint(1, 5)))


def build_pair(r, n_subs, n_clients, n_inline=0, fmt="spans"):
    e, o = EngineAdapter(fmt), OracleAdapter()
    for _ in range(n_subs):
        f = rand_filter(r)
        c = f"c{r.randrange(n_clients)}"
        kw = dict(qos=r.randint(0, 2), identifier=r.choice([0, 0, 3, 9, 200]),
                  no_local=r.random() < 0.2, rap=r.random() < 0.5, rh=r.randint(0, 2))
        assert e.subscribe(c, f, **kw) == o.subscribe(c, f, **kw)
    for _ in range(n_inline):
        f, i = rand_filter(r), r.randint(1, 6)
        assert e.inline_subscribe(f, i) == o.inline_subscribe(f, i)
    return e, o


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("seed", range(8))
def test_random_small_parity(seed, fmt, gpu_available):
    r = random.Random(1000 + seed)
    e, o = build_pair(r, 300, 12, n_inline=40, fmt=fmt)
    topics = ["/".join(r.choice(TSEGS) for _ in range(r.randint(1, 6))) for _ in range(400)]
    topics += ["", "a", "a/", "/", "//", "$SYS", "a/+", "+", "#", "a/#", "+/+", "a/b/c/+/#"]
    got = e.subscribers_batch(topics)
    for t, g in zip(topics, got):
        assert g == o.subscribers(t), t


def test_single_topic_batches_and_empty_batch(gpu_available):
    e, o = build_pair(random.Random(5), 100, 5)
    for t in ["a/b", "", "$SYS/x", "sport/a"]:
        assert e.subscribers(t) == o.subscribers(t), t
    assert e.subscribers_batch([]) == []


def test_deep_and_long_topics(gpu_available):
    e, o = EngineAdapter(), OracleAdapter()
    deep = "/".join(f"l{i}" for i in range(60))
    for f in [deep, deep[:200] + "/#", "/".join(["+"] * 60), "l0/#", "#",
              "x" * 300, "x" * 300 + "/+", "a/" + "y" * 1000]:
        for c in ("c1", "c2"):
            assert e.subscribe(c, f, identifier=len(f) % 7) == o.subscribe(c, f, identifier=len(f) % 7)
    topics = [deep, deep[:200], "/".join(f"l{i}" for i in range(61)), "x" * 300, "x" * 300 + "/q",
              "x" * 299, "a/" + "y" * 1000, "a/" + "y" * 999 + "z"]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t[:40]


def test_long_segment_hash_verification(gpu_available):
    """Segments > 15 bytes are hashed; a hit is verified byte for byte (no false matches)."""
    e, o = EngineAdapter(), OracleAdapter()
    base = "s" * 40
    for i in range(50):
        f = base + str(i) + "/v"
        e.subscribe("c", f)
        o.subscribe("c", f)
    topics = [base + str(i) + "/v" for i in range(60)] + [base + "x/v", base[:-1] + "/v"]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


def test_unicode_share_prefix(gpu_available):
    e, o = EngineAdapter(), OracleAdapter()
    for f in ["$ſhare/g/a/b", "$SHARE/g/a/b", "$share/h/a/+", "$Share/g/a/#", "$ſhar/g/a/b",
              "$sharE/g", "$share"]:
        assert e.subscribe("c1", f) == o.subscribe("c1", f)
        assert e.subscribe("c2", f) == o.subscribe("c2", f)
    for t in ["a/b", "a", "g", "$share", "$ſhar/g/a/b"]:
        assert e.subscribers(t) == o.subscribers(t), t


def test_inline_last_write_wins(gpu_available):
    e, o = EngineAdapter(), OracleAdapter()
    for f, i in [("a/b", 1), ("a/+", 1), ("#", 1), ("a/#", 2), ("+/b", 2), ("a/b", 3), ("a/b/#", 3)]:
        assert e.inline_subscribe(f, i) == o.inline_subscribe(f, i)
    for t in ["a/b", "a", "a/b/c", "x/b", "$SYS/b"]:
        assert e.subscribers(t) == o.subscribers(t), t


def test_dollar_rule_shared_and_inline_not_excluded(gpu_available):
    """Q3: the '$' rule drops only non-shared subscriptions whose filter starts with a wildcard."""
    e, o = EngineAdapter(), OracleAdapter()
    for c, f in [("c1", "#"), ("c2", "+/info"), ("c3", "$share/g/#"), ("c4", "$share/g/+/info"),
                 ("c5", "$SYS/#"), ("c6", "+abc/info")]:
        e.subscribe(c, f)
        o.subscribe(c, f)
    e.inline_subscribe("#", 9)
    o.inline_subscribe("#", 9)
    for t in ["$SYS/info", "$foo/info", "x/info", "+abc/info"]:
        assert e.subscribers(t) == o.subscribers(t), t


def _workload_pair(n_subs, n_clients, seed):
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(n_subs, n_clients, seed=seed)
    eng = E.Engine()
    orc = O.OracleIndex()
    assert (eng.subscribe_bulk(w) == orc.subscribe_bulk(w)).all()
    return w, eng, orc


def _digest_parity(eng, orc, tb, to, fmts=("rows", "spans")):
    """Per-topic digests of the engine in each result format against the oracle's."""
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
    for fmt in fmts:
        res = eng.match_batch_spans(tb, to) if fmt == "spans" else eng.match_batch(tb, to)
        dg, cnt = engine_digests(res)
        bad = np.nonzero(dg != od)[0]
        assert len(bad) == 0, (f"{fmt}: {len(bad)} topics differ, first {bad[:5]}, counts {cnt[bad[:3]]} vs "
                               f"{ocnt[bad[:3]]}")
        if fmt == "spans":  # the patches name a small part of the rows; each row at most once
            assert res["n_patches"] <= int(res["sub_cap"].sum())
    return cnt


@pytest.mark.parametrize("n_subs,n_clients,n_topics", [(10000, 1000, 20000), (200000, 20000, 20000),
                                                     (1000000, 100000, 6000)])
def test_workload_digest_parity(n_subs, n_clients, n_topics, gpu_available):
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(n_subs, n_clients, seed=11)
    tb, to = W.gen_topics(w, n_topics, seed=12)
    cnt = _digest_parity(eng, orc, tb, to)
    assert cnt[:, 0].sum() > n_topics  # the workload really fans out


def test_iot_workload_parity(gpu_available):
    from mqmatch import workload as W
    w = W.gen_subscriptions(50000, 50000, seed=21, mix=W.MIX_IOT)
    from mqmatch import engine as E
    eng, orc = E.Engine(), O.OracleIndex()
    eng.subscribe_bulk(w)
    orc.subscribe_bulk(w)
    tb, to = W.gen_topics(w, 20000, seed=22, mix=W.MIX_IOT)
    _digest_parity(eng, orc, tb, to)


def test_incremental_updates_between_batches(gpu_available):
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(30000, 3000, seed=31)
    tb, to = W.gen_topics(w, 5000, seed=32)
    _digest_parity(eng, orc, tb, to)
    fs = W.strings(w["bytes"], w["offs"])
    r = random.Random(33)
    for _ in range(3):
        for _ in range(2000):  # unsubscribe / resubscribe / new subscriptions
            i = r.randrange(len(fs))
            c = int(w["client_ids"][i])
            if r.random() < 0.5:
                assert bool(eng.unsubscribe(fs[i], c)) == orc.unsubscribe(fs[i], f"c{c:07d}")
            else:
                c2 = r.randrange(3000)
                fid = int(w["filter_ids"][i])
                a = eng.subscribe(fs[i], c2, fid, 1, 0, 7)
                b = orc.subscribe(f"c{c2:07d}", fs[i], 1, 7, client_id=c2, filter_id=fid)
                assert bool(a) == b
        st = eng.stats()
        _digest_parity(eng, orc, tb, to)
    assert st["upload_bytes_total"] > 0


def test_chunked_outputs(gpu_available):
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(50000, 5000, seed=41)
    eng.set_option(E.OPT_CHUNK_ROWS, 200000)
    tb, to = W.gen_topics(w, 30000, seed=42)
    _digest_parity(eng, orc, tb, to, fmts=("rows",))
    assert eng.match_chunks() > 1


def test_subbatch_pipeline(gpu_available):
    """Batches cut into pipelined sub-batches (walk of sub-batch b + 1 under the copies of b),
    each with several output chunks: results identical to the oracle."""
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(50000, 5000, seed=43)
    tb, to = W.gen_topics(w, 30000, seed=44)
    eng.set_option(E.OPT_SUBBATCH_TOPICS, 4096)
    eng.set_option(E.OPT_CHUNK_ROWS, 300000)
    _digest_parity(eng, orc, tb, to, fmts=("rows",))
    assert eng.match_chunks() >= 8
    eng.set_option(E.OPT_SUBBATCH_TOPICS, 1024)  # one scan block per sub-batch
    _digest_parity(eng, orc, tb, to[:5001], fmts=("rows",))


def test_subbatch_gather_overflow(gpu_available):
    """Gather-slot overflow (compact fill pass) in some sub-batches only."""
    e, o = EngineAdapter("rows"), OracleAdapter()
    e.x.engine.set_option(e.E.OPT_SUBBATCH_TOPICS, 1024)
    levels = [f"l{i}" for i in range(80)]
    for d in range(1, 80):
        f = "/".join(levels[:d]) + "/#"
        assert e.subscribe(f"c{d % 7}", f, identifier=d) == o.subscribe(f"c{d % 7}", f, identifier=d)
    deep = "/".join(levels)
    topics = [f"l0/x{i}" for i in range(3000)] + [deep] * 3 + ["/".join(levels[:5])] * 2000
    got = e.subscribers_batch(topics)
    for t in (topics[0], deep, topics[-1]):
        assert got[topics.index(t)] == o.subscribers(t), t
    assert got[3000] == got[3002]


@pytest.mark.parametrize("fmt", FORMATS)
def test_long_lists_with_merges(fmt, gpu_available):
    """Lists of thousands of subscriptions (root '#', 'a/#': one span each, or many k_copy tiles
    over one list) in which some clients hold co-matching filters, so merge bases and ident rows
    sit inside long lists."""
    e, o = EngineAdapter(fmt), OracleAdapter()
    for i in range(3000):
        c = f"h{i}"
        assert e.subscribe(c, "#", qos=i % 3, identifier=i % 5) == o.subscribe(c, "#", qos=i % 3, identifier=i % 5)
        if i % 2:
            assert e.subscribe(c, "a/#", identifier=i % 7) == o.subscribe(c, "a/#", identifier=i % 7)
        if i % 5 == 0:
            assert e.subscribe(c, "a/+/c", qos=2) == o.subscribe(c, "a/+/c", qos=2)
    for i in range(1500):
        c = f"k{i}"
        assert e.subscribe(c, "a/b/c") == o.subscribe(c, "a/b/c")
    topics = (["a/b/c", "a/x", "b", "$SYS/x", "a", "a/b/c/d"] * 50)[:300]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


def test_match_device_chunks_consumer(gpu_available):
    """mq_match_device_chunks: a consumer copying every chunk to the host on the chunk stream
    sees exactly mq_match_batch's rows and per-topic records."""
    import ctypes as C
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(50000, 5000, seed=45)
    eng.set_option(E.OPT_CHUNK_ROWS, 150000)
    tb, to = W.gen_topics(w, 20000, seed=46)
    n = len(to) - 1
    host = eng.match_batch(tb, to)
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    hip.hipMemcpyAsync.restype = C.c_int
    rows = np.zeros((len(host["rows"]), 4), np.uint32)
    topics = np.zeros((n, 12), np.uint32)
    bases = []

    def consume(chunk, first, stream):
        r0 = sum(c for _, _, c in bases)
        if chunk.n_sub_rows:
            assert hip.hipMemcpyAsync(rows[r0:].ctypes.data, chunk.sub_rows, chunk.n_sub_rows * 16, 2, stream) == 0
        assert hip.hipMemcpyAsync(topics[first:].ctypes.data, chunk.topics, chunk.n_topics * 48, 2, stream) == 0
        bases.append((first, chunk.n_topics, chunk.n_sub_rows))

    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    s = torch.cuda.Stream()
    eng.match_device_chunks(d_tb.data_ptr(), d_to.data_ptr(), n, s.cuda_stream, consume)
    torch.cuda.synchronize()
    assert len(bases) == eng.match_chunks() > 2
    assert (rows == host["rows"]).all()
    sub_base = topics[:, 0].astype(np.uint64) | (topics[:, 1].astype(np.uint64) << np.uint64(32))
    r0 = 0
    for first, nt, nr in bases:
        sub_base[first:first + nt] += np.uint64(r0)
        r0 += nr
    assert (sub_base == host["sub_base"]).all()
    assert (topics[:, 6] == host["sub_cap"]).all() and (topics[:, 7] == host["n_client"]).all()
    assert (topics[:, 8] == host["n_ident"]).all() and (topics[:, 10] == host["n_inline"]).all()


def test_match_device_stream(gpu_available):
    """mq_match_device on torch-owned device buffers and a torch stream."""
    import torch
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(20000, 2000, seed=51)
    tb, to = W.gen_topics(w, 4096, seed=52)
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        r = eng.match_device(d_tb.data_ptr(), d_to.data_ptr(), len(to) - 1, s.cuda_stream)
    s.synchronize()
    host = eng.match_batch(tb, to)
    assert r.n_topics == len(to) - 1 and r.n_sub_rows == len(host["rows"])


def test_spans_patch_pool_growth(gpu_available):
    """A patch pool far smaller than a batch needs: the batch's reservations exceed it, the pool
    grows and k_merge runs again; the result is unchanged."""
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(60000, 3000, seed=47)
    eng.set_option(E.OPT_PATCH_CAP, 64)
    tb, to = W.gen_topics(w, 8000, seed=48)
    _digest_parity(eng, orc, tb, to, fmts=("spans",))
    _digest_parity(eng, orc, tb, to, fmts=("spans",))  # the grown pool is kept


@pytest.mark.parametrize("codes", [1, 0])
def test_host_spans_first_batch_outgrows_pools(codes, gpu_available):
    """The first batch of a fresh index, host results, with patch pools far too small (64 slots):
    its one-sync run overflows both pools, so the packing kernels that run before the batch's
    readback must copy nothing from a set whose reservation did not fit (a regression: k_set_pack
    copied such sets' counts past the pool and the stage). Pipelined submit first, then a plain
    host match; both equal the oracle."""
    import ctypes as C
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(200000, 20000, seed=83)
    eng.set_option(E.OPT_PATCH_CAP, 64)
    eng.set_option(E.OPT_PATCH_CODES, codes)
    tb, to = W.gen_topics(w, 30000, seed=84)
    n = len(to) - 1
    want = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))[0]
    t = C.c_void_p()
    E._check(E.lib().mq_match_spans_submit(eng.h, E._p(tb, E._u8p), E._p(to, E._u64p), n, C.byref(t)), "submit")
    rp = C.POINTER(E.SpanResult)()
    E._check(E.lib().mq_match_spans_wait(t, C.byref(rp)), "wait")
    assert (engine_digests(E._expand_host_spans(rp, n))[0] == want).all()
    _digest_parity(eng, orc, tb, to, fmts=("spans",))


def test_spans_format_shape(gpu_available):
    """The span format itself: spans in gather order cover exactly n_rows records, patch rows are
    in range and unique per topic, and a topic without co-matching records has no patches."""
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(40000, 4000, seed=49)
    tb, to = W.gen_topics(w, 3000, seed=50)
    a = eng.match_spans(tb, to)
    t, spans = a["topics"], a["spans"]
    tid, prow, pmeta = E.host_topic_patches(a)
    assert len(tid) == int(t["n_patches"].sum())
    for i in range(len(t)):
        sp = spans[int(t["span_base"][i]):int(t["span_base"][i]) + int(t["n_spans"][i])]
        assert int(sp[:, 1].sum()) == int(t["n_rows"][i])
        assert int(sp[:, 3].sum()) == int(t["n_shared"][i])
        pr, pm = prow[tid == i], pmeta[tid == i]
        assert len(set(pr.tolist())) == len(pr) and (pr < max(1, int(t["n_rows"][i]))).all()
        if int(t["n_client"][i]) == int(t["n_rows"][i]):
            assert ((pm & 0xC0000000) == 0).all()
    # host results share merge-set patches as device results do (ABI v7)
    assert ((t["flags"] & 1) != 0).any() and len(a["merge_base"]) == len(t)
    rows_bytes = 16 * int(t["n_rows"].sum())
    span_bytes = (64 * len(t) + 16 * len(spans) + 8 * len(a["patches"]) + 8 * len(a["set_patches"])
                  + 4 * len(a["merge_rows"]) + 4 * len(a["merge_base"]))
    assert span_bytes * 4 < rows_bytes  # the point of the format


@pytest.mark.parametrize("dedup,codes", [(0, 1), (1, 1), (0, 0), (1, 0)])
def test_host_spans_own_and_set_patches(dedup, codes, gpu_available):
    """Host span results (mq_match_spans) with merge-set dedup (topics name their set's packed
    patches through their packed merge rows) and without (every topic's own packed patches), with
    4-byte patch codes (MQ_SPANS_PATCH_CODES, the default) and 8-byte patches: expanded rows equal
    the oracle's, and the patch arrays are what the mode says."""
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(40000, 3000, seed=71)
    eng.set_option(E.OPT_MERGE_DEDUP, dedup)
    eng.set_option(E.OPT_PATCH_CODES, codes)
    tb, to = W.gen_topics(w, 4000, seed=72)
    _digest_parity(eng, orc, tb, to, fmts=("spans",))
    a = eng.match_spans(tb, to)
    assert a["patch_codes"] == bool(codes)
    setf = (a["topics"]["flags"] & 1) != 0
    if dedup:
        assert setf.any() and len(a["set_patches"]) > 0 and len(a["merge_base"]) == len(setf)
    else:
        assert not setf.any() and len(a["set_patches"]) == 0 and len(a["patches"]) > 0
    tid, prow, _ = E.host_topic_patches(a)
    assert len(tid) == int(a["topics"]["n_patches"].sum()) and (prow < a["topics"]["n_rows"][tid]).all()


def test_spans_pipelined_batches(gpu_available):
    """Pipelined host results (mq_match_spans_submit / _wait, ABI v8): consecutive batches of
    different sizes (an empty one, small ones, one several times larger than the others, so its
    buffers are outgrown and it runs again), each waited for after the next is submitted — so a
    batch's copy into host memory runs while the next batch's kernels write the other stage —
    expand to the oracle's digests; an update between submits shows in the later batches only."""
    import ctypes as C
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(40000, 3000, seed=73)
    sizes = [3000, 0, 500, 12000, 3000, 1]
    batches = [W.gen_topics(w, k, seed=74 + i) if k else (np.zeros(16, np.uint8), np.zeros(1, np.uint64))
               for i, k in enumerate(sizes)]
    want = [orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))[0] for tb, to in batches]

    def submit(tb, to):
        t = C.c_void_p()
        assert E.lib().mq_match_spans_submit(eng.h, E._p(tb, E._u8p), E._p(to, E._u64p), len(to) - 1,
                                             C.byref(t)) == 0
        return t

    def wait(t, n):
        rp = C.POINTER(E.SpanResult)()
        assert E.lib().mq_match_spans_wait(t, C.byref(rp)) == 0
        return E._expand_host_spans(rp, n)

    for rnd in range(2):  # (the second round: every stage and buffer sized already)
        pend = []
        for i, (tb, to) in enumerate(batches):
            pend.append((i, submit(tb, to)))
            if len(pend) == 2:
                j, t = pend.pop(0)
                dg, _ = engine_digests(wait(t, len(batches[j][1]) - 1))
                assert (dg == want[j]).all(), (rnd, j)
        for j, t in pend:
            dg, _ = engine_digests(wait(t, len(batches[j][1]) - 1))
            assert (dg == want[j]).all(), (rnd, j)
    # an update between two submits: the first result is the index before it, the second after
    tb, to = W.gen_topics(w, 2000, seed=90)
    t0 = submit(tb, to)
    before = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))[0]
    # (a plain update; mq_subscribe_bulk behaves the same: test_bulk_subscribe_beside_pipelined). A new client on
    # the root '#' list every topic gathers (its filter id is the workload's id of "#": ids name
    # filter strings)
    offs = w["offs"].astype(np.int64)
    fid = next(int(w["filter_ids"][i]) for i in range(len(offs) - 1) if bytes(w["bytes"][offs[i]:offs[i + 1]]) == b"#")
    assert eng.subscribe("#", 999999, fid, 2, 0, 0) == int(orc.subscribe("c999999", "#", qos=2, client_id=999999,
                                                                          filter_id=fid))
    after = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))[0]
    t1 = submit(tb, to)
    assert (engine_digests(wait(t0, 2000))[0] == before).all()
    assert (engine_digests(wait(t1, 2000))[0] == after).all()
    assert not (before == after).all()


def test_bulk_subscribe_beside_pipelined(gpu_available):
    """A restore (mq_subscribe_bulk) while pipelined tickets are outstanding does not wait for them
    (submit k+1 waited for the bulk update, which waited for ticket k's result — a
    deadlock). Run on a worker thread with a deadline: an empty index with a live ticket takes the
    per-entry path; the ticket shows the index before, the next submit the index after, both
    equal to the oracle; the bulk results equal the oracle's."""
    import threading
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(30000, 3000, seed=95)
    eng, orc = E.Engine(device=0), O.OracleIndex()
    tb, to = W.gen_topics(w, 2000, seed=96)
    out = {}

    def body():
        rc, t0 = _submit(eng, tb, to)
        assert rc == 0
        out["bulk"] = eng.subscribe_bulk(w)  # (the ticket's result is live: per-entry, copy-on-write)
        rc, t1 = _submit(eng, tb, to)
        assert rc == 0
        out["r0"] = _wait(t0, 2000)
        out["r1"] = _wait(t1, 2000)

    th = threading.Thread(target=body, daemon=True)
    th.start()
    th.join(timeout=90)
    assert not th.is_alive(), "bulk subscribe beside an outstanding ticket did not finish"
    empty = O.OracleIndex().digest_batch(tb, to, nthreads=4)[0]
    assert (out["bulk"] == orc.subscribe_bulk(w)).all()
    full = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))[0]
    assert out["r0"][0] == 0 and (engine_digests(out["r0"][1])[0] == empty).all()
    assert out["r1"][0] == 0 and (engine_digests(out["r1"][1])[0] == full).all()
    eng.check()


def test_spans_device_matches_host(gpu_available):
    """mq_match_spans_device on torch buffers: the same per-topic records as mq_match_spans."""
    import ctypes as C
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(20000, 2000, seed=53)
    tb, to = W.gen_topics(w, 4096, seed=54)
    host = eng.match_spans(tb, to)
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    s = torch.cuda.Stream()
    r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), len(to) - 1, s.cuda_stream)
    n = len(to) - 1
    top = torch.empty(n * 16, dtype=torch.int32, device="cuda")
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(top.data_ptr(), r.topics, n * 64, 3) == 0
    got = top.cpu().numpy().view(E._TOPIC_SPANS_DT)
    for k in ("n_spans", "n_rows", "n_client", "n_ident", "n_shared", "n_inline", "n_patches"):
        assert (got[k] == host["topics"][k]).all(), k
    # the same spans per topic (a one-sync device batch places topic t's at t * 64: the walk-fused
    # desc's stride layout; host results are packed)
    sb, ns = got["span_base"].astype(np.int64), got["n_spans"].astype(np.int64)
    ext = int((sb + ns).max())
    own = (host["topics"]["flags"] & 1) == 0
    assert (got["flags"] == host["topics"]["flags"]).all()
    assert r.n_spans >= ext and r.n_patches >= int(host["topics"]["n_patches"][own].sum())
    dsp = torch.empty(ext * 4, dtype=torch.int32, device="cuda")
    assert hip.hipMemcpy(dsp.data_ptr(), r.spans, ext * 16, 3) == 0
    dsp = dsp.cpu().numpy().view(np.uint32).reshape(-1, 4)
    ht = host["topics"]  # (host spans are packed, each topic's run at its span_base, in no set order)
    hsp = host["spans"][E._ranges(ht["span_base"].astype(np.int64), ht["n_spans"].astype(np.int64))]
    assert (dsp[E._ranges(sb, ns)] == hsp).all()


@pytest.mark.parametrize("exp,waves", [(0, 8), (16 | 128, 8), (32 | 128, 8), (64 | 128, 8), (0, 7), (0, 6),
                                       (128, 8), (256, 8), (512, 8), (256 | 512, 8)])
def test_set_pass_variants_exact(exp, waves, gpu_available):
    """The merge set pass's exact variants: the fold (default: records folded over their visits, no
    partner links), bit 7 (records resolved through their partner links), with bit 4 (a visit
    through a partner other than the record's first reads all its links) or bits 5 / 6 (3 / 4
    partner links per batch); bit 8 (fold chunks of 16 visits: many chunks per set, and merge
    gathers beyond a chunk take the record-indexed bit fold); bit 9 (merge gathers too big for the
    hash fold resolved through their partner links, as before round 5); 7 or 6 waves per SIMD
    (MQ_OPT_MERGE_WAVES): per-topic digests of device results equal the oracle's."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(60000, 3000, seed=65)
    eng.set_option(E.OPT_SET_EXP, exp)
    eng.set_option(E.OPT_MERGE_WAVES, waves)
    tb, to = W.gen_topics(w, 6000, seed=66)
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    torch.cuda.synchronize()
    od, _, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
    for _ in range(2):  # (the second batch: one synchronisation, sized by the first)
        r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
        res = E.expand_device_spans(r, n)
        assert res["set_topics"] > 0
        dg, _ = engine_digests(res)
        bad = np.nonzero(dg != od)[0]
        assert len(bad) == 0, f"{len(bad)} of {n} topics differ (first {bad[:5]})"


@pytest.mark.parametrize("dedup,fuse,group", [(1, 1, 16), (1, 0, 16), (0, 1, 16), (1, 1, 0)])
def test_spans_device_digest_parity(dedup, fuse, group, gpu_available):
    """mq_match_spans_device expanded as a device consumer would (spans, then per-topic patches or
    set-shared patches through the topic's merge rows, inline rows): per-topic digests equal the
    oracle's. With merge-set dedup (the default) topics share their merge set's patches
    (MQ_TOPIC_SET_PATCHES); without it every topic holds its own. fuse: k_desc in the walk's
    epilogue (the stride layout of one-sync batches, MQ_OPT_FUSE_DESC) or walk, scan, k_desc."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(60000, 3000, seed=63)
    eng.set_option(E.OPT_MERGE_DEDUP, dedup)
    eng.set_option(E.OPT_FUSE_DESC, fuse)
    eng.set_option(E.OPT_WALK_GROUP, group)  # 0: the walk thread per topic (+ scan + k_desc)
    tb, to = W.gen_topics(w, 6000, seed=64)
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    torch.cuda.synchronize()
    r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
    res = E.expand_device_spans(r, n)
    assert (res["set_topics"] > 0) == bool(dedup)
    dg, cnt = engine_digests(res)
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
    bad = np.nonzero(dg != od)[0]
    assert len(bad) == 0, f"{len(bad)} of {n} topics differ (first {bad[:5]})"


@pytest.mark.parametrize("group", [16, 0])
def test_walk_same_segment_many_parents(group, gpu_available):
    """Thousands of particles share the segment "a" under other parents, so probe runs hold
    slots of the topic's own segment under foreign parents before (or instead of) the topic's
    edge; long (hashed) segments and a '+' level are mixed in, and the edge table runs at load
    1/2 for longer probe runs. Both walks (the frontier walk, the walk thread per topic)."""
    from mqmatch import engine as E
    e, o = EngineAdapter(), OracleAdapter()
    e.x.engine.set_option(E.OPT_EDGE_LOAD, 2)
    e.x.engine.set_option(E.OPT_WALK_GROUP, group)
    long = "s" * 40
    subs = []
    for i in range(3000):
        subs += [(f"c{i % 97}", f"p{i}/a"), (f"d{i % 89}", f"p{i}/a/a/#")]
        if i % 3 == 0:
            subs.append((f"e{i % 13}", f"p{i}/+/a/{long}"))
        if i % 5 == 0:
            subs.append((f"f{i % 7}", "+/a/a/a"))
    for c, f in subs:
        assert e.subscribe(c, f, identifier=len(f) % 3) == o.subscribe(c, f, identifier=len(f) % 3)
    topics = ([f"p{i}/a" for i in range(0, 3000, 7)] + [f"q{i}/a" for i in range(300)] +
              [f"p{i}/a/a/a" for i in range(0, 3000, 11)] + [f"p{i}/x/a/{long}" for i in range(0, 3000, 9)] +
              [f"p{i}/+/a/{long}" for i in range(0, 300, 9)] + [f"p{i}/a/a/a/a/a" for i in range(0, 3000, 13)])
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


def test_walk_nested_plus_paths(gpu_available):
    """Every literal/'+' path of depth 5 and 6 subscribed (and their '#' parents), so a topic's
    frontier is as wide as it gets at each level (beyond the frontier's 16 particles the topic
    goes to the walk thread per topic)."""
    import itertools
    e, o = EngineAdapter(), OracleAdapter()
    for depth in (5, 6):
        for k, bits in enumerate(itertools.product((0, 1), repeat=depth)):
            f = "/".join(f"a{i}" if b == 0 else "+" for i, b in enumerate(bits))
            assert e.subscribe(f"c{k % 50}", f, identifier=k % 4) == o.subscribe(f"c{k % 50}", f, identifier=k % 4)
            if k % 3 == 0:
                f2 = "/".join(f"a{i}" if b == 0 else "+" for i, b in enumerate(bits[:-1])) + "/#"
                assert e.subscribe(f"h{k % 7}", f2) == o.subscribe(f"h{k % 7}", f2)
    topics = ["/".join(f"a{i}" for i in range(d)) for d in range(1, 8)] + ["a0/x/a2/a3/x", "x/x/x/x/x/x"]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


def test_walk_trials_choose_and_stay_exact(gpu_available):
    """Device batches of 64k+ topics time both walks on their first batches (the frontier walk with
    the fused desc, the walk thread per topic with scan + desc) and keep the faster: every batch,
    trial or not, equals the oracle, and both trials ran."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(20000, 2000, seed=81)
    tb, to = W.gen_topics(w, 70000, seed=82)
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    od, _, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
    eng.profile(True)
    for _ in range(8):  # (6 trial batches: one untimed per walk, then two timed per walk, ABBA)
        torch.cuda.synchronize()
        r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
        dg, _ = engine_digests(E.expand_device_spans(r, n))
        assert (dg == od).all()
    prof = eng.profile_read()
    assert "trial_frontier_ps_per_topic" in prof and "trial_thread_ps_per_topic" in prof, sorted(prof)
    assert prof["trial_frontier_batches"][0] == 2 and prof["trial_thread_batches"][0] == 2
    assert ("trial_chose_thread" in prof) != ("trial_chose_frontier" in prof)


def test_walk_trials_rearm_on_wildcard_mix(gpu_available):
    """The walk trials run again when the index's wildcard mix moves without its size doubling:
    an exact-match (IoT) index runs its trials, then wildcard-heavy subscriptions join (the share
    of '+' / '#' particles rises well past a quarter of itself), and the next batches time both
    walks again; every batch equals the oracle."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(30000, 30000, seed=91, mix=W.MIX_IOT)
    eng, orc = E.Engine(), O.OracleIndex()
    assert (eng.subscribe_bulk(w) == orc.subscribe_bulk(w)).all()
    w2 = W.gen_subscriptions(6000, 600, seed=92)  # (the mqtt mix: wildcard-heavy)

    def batches(wt, seed, k):
        tb, to = W.gen_topics(wt, 70000, seed=seed)
        n = len(to) - 1
        d_tb = torch.from_numpy(tb).cuda()
        d_to = torch.from_numpy(to.view(np.int64)).cuda()
        od, _, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
        eng.profile(True)
        eng.profile_reset()
        for _ in range(k):
            torch.cuda.synchronize()
            r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
            dg, _ = engine_digests(E.expand_device_spans(r, n))
            assert (dg == od).all()
        return eng.profile_read()

    prof = batches(w, 93, 6)
    assert "trial_frontier_ps_per_topic" in prof and "trial_thread_ps_per_topic" in prof, sorted(prof)
    assert ("trial_chose_thread" in prof) != ("trial_chose_frontier" in prof)
    prof = batches(w, 94, 2)
    assert "trial_frontier_ps_per_topic" not in prof  # same index: the choice stays
    nodes0 = eng.stats().get("nodes")
    assert (eng.subscribe_bulk(w2) == orc.subscribe_bulk(w2)).all()
    nodes1 = eng.stats().get("nodes")
    assert nodes0 is None or nodes1 < 2 * nodes0  # (not a new size: a new mix)
    prof = batches(w2, 95, 6)
    assert "trial_frontier_ps_per_topic" in prof and "trial_thread_ps_per_topic" in prof, sorted(prof)


@pytest.mark.parametrize("fuse", [0, 1])
def test_one_sync_batches_grow_and_repeat(fuse, gpu_available):
    """One-sync batches (MQ_OPT_ONE_SYNC, the default for device results): buffers sized by
    earlier batches. A fresh index, a small batch, then a batch several times larger (its spans
    and patches do not fit what the small one left: it runs again, sized by the host), then the
    large batch again (fits: one synchronisation) and the small one: every result equals the
    oracle's, and the profile counts exactly the runs that had to repeat. With k_desc fused into
    the walk (MQ_OPT_FUSE_DESC, the default) the spans' stride layout is sized by the batch
    itself, so only a gather-slot overflow repeats a run."""
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(60000, 3000, seed=71)
    eng.set_option(E.OPT_FUSE_DESC, fuse)
    eng.profile(True)
    batches = [W.gen_topics(w, k, seed=72 + i) for i, k in enumerate((300, 6000))]
    retried = []
    for tb, to in (batches[0], batches[1], batches[1], batches[0]):
        n = len(to) - 1
        d_tb = torch.from_numpy(tb).cuda()
        d_to = torch.from_numpy(to.view(np.int64)).cuda()
        torch.cuda.synchronize()
        eng.profile_reset()
        r = eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
        prof = eng.profile_read()
        # a topic with more gathers than its slot (walk_fill in the host-sized run) always repeats
        retried.append((prof.get("one_sync_retries", (0, 0.0))[0], "walk_fill" in prof))
        dg, _ = engine_digests(E.expand_device_spans(r, n))
        od, _, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
        assert (dg == od).all()
    # unfused: the first batch (nothing sized yet) and the first large one repeat; the others
    # only for a slot overflow
    first = (1, 1) if not fuse else (int(retried[0][1]), int(retried[1][1]))
    assert [x[0] for x in retried] == [*first, int(retried[2][1]), int(retried[3][1])], retried


def test_spans_result_survives_updates(gpu_available):
    """A host span result points into the host image's subscription pools until it is freed;
    updates do not wait for it (capi.cpp IndexLock): the index copies a slab before it changes one
    a live result may see and keeps freed slabs and outgrown pool buffers until no live result
    can see them. While results are held, the same thread and another one overwrite, remove,
    flip may-merge slots, add shared members and grow both pools past their capacity; each held
    result still expands to exactly what it matched, and the image stays consistent."""
    import ctypes as C
    import threading
    from mqmatch import engine as E
    eng = E.Engine()
    for c in range(50):
        eng.subscribe("a/+", c, 0, 1, 0, 0)
        eng.subscribe("a/b", 200 + c, 1, 0, 0, 0)
    for c in range(12):
        eng.subscribe("$share/g/a/+", 400 + c, 2, 0, 0, 0)
    tb, to = E.pack_strings(["a/b", "a/c", "x"])

    def held():
        rp = C.POINTER(E.SpanResult)()
        assert E.lib().mq_match_spans(eng.h, E._p(tb, E._u8p), E._p(to, E._u64p), 3, C.byref(rp)) == 0
        return rp

    def same(a, b):
        for k in ("rows", "shared", "sub_cap", "n_client", "n_shared"):
            assert np.array_equal(a[k], b[k]), k

    want0 = eng.match_batch_spans(tb, to)
    r0 = held()
    # in place: overwrite (qos), remove from the middle, flip slots to may-merge and back
    for c in range(0, 50, 3):
        assert eng.subscribe("a/+", c, 0, 2, 0, 0) == 0
    for c in range(1, 50, 4):
        assert eng.unsubscribe("a/+", c) == 1
    for c in range(0, 50, 5):
        eng.subscribe("a/#", c, 3, 0, 0, 0)
    for c in range(0, 50, 10):
        eng.unsubscribe("a/#", c)
    for c in range(0, 12, 2):
        eng.subscribe("$share/g/a/+", 400 + c, 7, 0, 0, 0)
    eng.unsubscribe("$share/g/a/+", 401)
    want1 = eng.match_batch_spans(tb, to)
    r1 = held()
    # from another thread, while r0 and r1 are held: grow both pools past their capacity
    done = []

    def grow():
        for c in range(3000):
            eng.subscribe("a/+", 1000 + c, 0, 0, 0, 0)
            eng.subscribe("$share/h/a/b", 5000 + c, 8, 0, 0, 0)
            eng.subscribe("f/%d" % c, c, 9, 0, 0, 0)
        done.append(1)
    th = threading.Thread(target=grow)
    th.start()
    th.join(timeout=120)
    assert done == [1]  # did not wait for the held results
    eng.check()
    same(E._expand_host_spans(r0, 3), want0)  # (frees r0)
    same(E._expand_host_spans(r1, 3), want1)
    for c in range(3000):  # the slabs kept for r0 / r1 go back to the pools
        eng.unsubscribe("f/%d" % c, c)
    eng.check()
    got = eng.match_batch_spans(tb, to)
    plus = set(range(50)) - set(range(1, 50, 4)) | set(range(1000, 4000))
    clients = plus | set(range(200, 250)) | set(range(5, 50, 10))  # a/+, a/b, a/#
    assert int(got["n_client"][0]) == len(clients)
    assert int(got["n_shared"][0]) == (12 - 1) + 3000  # members of $share/g/a/+ and $share/h/a/b


MSEGS = ["a", "b", "c", "", "$SYS", "$share", "g", "x", "averyveryverylongsegment", "ü", "$x"]


@pytest.mark.parametrize("image", [True, False])
@pytest.mark.parametrize("q6", [False, True])
@pytest.mark.parametrize("seed", range(6))
def test_messages_random_parity(seed, q6, image, gpu_available):
    """Messages (topics.go:525-579) on random retained sets, including Q4 ($SYS at level 0
    only), Q5 (x/# excludes x), Q6 (particles without a retain path; q6: a retained entry on
    topic "" is live, which the level-order image path hands to the particle walk), Q12 (expired
    entries). image: the level-order image (default) or the particle walk (MQ_OPT_MSG_IMAGE)."""
    r = random.Random(2000 + seed)
    topics = ["/".join(r.choice(MSEGS) for _ in range(r.randint(1, 5))) for _ in range(300)]
    topics = [t for t in topics if t != ""] + ([""] if q6 else [])
    e, o = EngineAdapter(msg_image=image), OracleAdapter()
    for i, t in enumerate(topics):
        pl = b"" if (r.random() < 0.1 and t != "") else b"p"
        ret = r.random() < 0.9
        a, _ = e.retain_message(t, pl, ret, handle=i + 1)
        b, _ = o.retain_message(t, pl, ret, handle=i + 1)
        assert a == b, t
    for t in topics[::13]:  # expiry sweep deletes map entries only (Q12)
        if t == "":
            continue
        e.retained_delete(t)
        o.retained_delete(t)
    for f in ["a/b", "q", "x/y"]:  # subscription-only particles (no retain path)
        e.subscribe("c", f)
        o.subscribe("c", f)
    filters = ["/".join(r.choice(MSEGS + ["+", "+", "#"]) for _ in range(r.randint(1, 5)))
               for _ in range(300)]
    filters += ["#", "+", "+/+", "$SYS/#", "$SYS/+", "a/#", "a/+/#", "", "a", "a/b", "#/a",
                "+/#", "a/#/b", "+/+/+", "+/a/+", "+/+/#", "$SYS", "+/$SYS/#"]
    got = e.messages_batch(filters)
    for f, g in zip(filters, got):
        assert g == o.messages(f), f


@pytest.mark.parametrize("image", [True, False])
def test_messages_after_retained_changes(image, gpu_available):
    """Retained changes between Messages batches (new topics, payload-less deletes, expiry
    sweeps, handle replacement): each batch sees the current state (the image is rebuilt)."""
    r = random.Random(77)
    e, o = EngineAdapter(msg_image=image), OracleAdapter()
    segs = ["a", "b", "c", "d", "$SYS", "x"]
    filters = ["#", "+", "+/+", "a/#", "+/b/#", "a/+", "+/+/+", "$SYS/#", "a/b", "+/c/+", "x/+/+/#"]
    handle = 0
    for round_ in range(8):
        for _ in range(60):
            t = "/".join(r.choice(segs) for _ in range(r.randint(1, 4)))
            u = r.random()
            handle += 1
            if u < 0.7:
                assert e.retain_message(t, b"p", True, handle=handle)[0] == \
                    o.retain_message(t, b"p", True, handle=handle)[0]
            elif u < 0.85:
                assert e.retain_message(t, b"", True, handle=handle)[0] == \
                    o.retain_message(t, b"", True, handle=handle)[0]
            else:
                e.retained_delete(t)
                o.retained_delete(t)
        got = e.messages_batch(filters)
        for f, g in zip(filters, got):
            assert g == o.messages(f), (round_, f)


@pytest.mark.parametrize("image", [True, False])
def test_retained_add_after_expiry(image, gpu_available):
    """Retained.Add outside RetainMessage (the Go shim's Retained wrapper, mq_retained_set) on
    topics whose particle keeps its retain path: an expired entry (Q12) re-added is found by
    wildcard and literal filters again, and RetainMessage's -1 answer reads the re-added packet."""
    from mqmatch import engine as E
    r = random.Random(5)
    e = E.Engine()
    if not image:
        e.set_option(E.OPT_MSG_IMAGE, 0)
    o = O.OracleIndex()
    segs = ["a", "b", "c", "$SYS"]
    path = set()  # topics whose particle has a retain path
    for step in range(600):
        t = "/".join(r.choice(segs) for _ in range(r.randint(1, 3)))
        u = r.random()
        h = step + 1
        if u < 0.5:
            pl = 0 if r.random() < 0.2 else 3
            ret = r.random() < 0.8
            assert e.retain_message(t, h, pl, ret) == o.retain_message(t, h, pl, ret), step
            (path.add if pl else path.discard)(t)
        elif u < 0.75:
            e.retained_delete(t)
            o.retained_delete(t)
        elif t in path:
            pl, ret = r.choice([0, 4]), r.random() < 0.5
            assert e.retained_set(t, h, pl, ret) == 1
            o.retained_add(t, h, pl, ret)
    assert e.retained_len() == o.retained_len()
    filters = ["#", "+", "+/+", "a/#", "+/b", "a/+/+", "$SYS/#"] + sorted(path)
    fb = "".join(filters).encode()
    offs = np.cumsum([0] + [len(f.encode()) for f in filters]).astype(np.uint64)
    bytes_ = np.frombuffer(fb + b"\0" * 16, np.uint8)
    base, count, hs = e.messages_batch(bytes_, offs)
    for i, f in enumerate(filters):
        got = sorted(hs[int(base[i]):int(base[i]) + int(count[i])].tolist())
        assert got == o.messages(f), f


def test_messages_deep_fanout(gpu_available):
    """A filter whose literal levels meet runs of two particles 18 times over nests fan-outs
    beyond a lane's frame stack (kMsgStack): the batch takes the particle walk, exactly."""
    e, o = EngineAdapter(), OracleAdapter()
    depth = 18
    h = 0
    for i in range(1, depth + 1):
        chain = "/".join(["p", "k"] * i)
        for t in (chain, chain[:-1] + "q", chain[:-3] + "q"):  # siblings at '+' levels
            h += 1
            e.retain_message(t, b"p", True, handle=h)
            o.retain_message(t, b"p", True, handle=h)
    filters = ["/".join(["+", "k"] * depth), "/".join(["+", "k"] * 3), "+/k/+/k/#", "#"]
    got = e.messages_batch(filters)
    for f, g in zip(filters, got):
        assert g == o.messages(f), f


@pytest.mark.parametrize("export,edges", [(1, 1), (0, 1), (1, 0)])
def test_messages_wide_fanout_export(export, edges, gpu_available):
    """Filters whose literal segment meets a fan-out of thousands of particles (w/+/c/...: 6,000
    children of w): the count pass hands those particles to work items every wavefront takes
    (MQ_OPT_MSG_EXPORT, kMsgExportMin) and their outputs land after the filter's own part. Mixed
    with small filters in one batch; equal to the oracle with and without the export, and with
    the literal lookups through the image's edge table (MQ_OPT_MSG_EDGES, the default) or the
    index's."""
    from mqmatch import engine as E
    e, o = EngineAdapter(), OracleAdapter()
    e.x.engine.set_option(E.OPT_MSG_EXPORT, export)
    e.x.engine.set_option(E.OPT_MSG_EDGES, edges)
    h = 0
    topics = []
    for i in range(6000):
        topics.append(f"w/{i}/c/{i % 3}")
        if i % 5 == 0:
            topics.append(f"w/{i}/d")
        if i % 7 == 0:
            topics.append(f"w/{i}/c/{i % 3}/e")
        if i % 2 == 0:
            topics.append(f"v/{i}/c/x")
    for t in topics + ["w/c", "q/r", "$SYS/w/1"]:
        h += 1
        assert e.retain_message(t, b"p", True, handle=h) == o.retain_message(t, b"p", True, handle=h)
    filters = ["w/+/c/+", "w/+/c/#", "w/+/d", "w/+/c/1", "+/+/c/+", "+/+/c/x", "w/+/c/+/e", "+/+/c/#",
               "v/+/c/+", "w/#", "q/+", "#", "w/1/c/1", "+/17/c/+"]
    filters = filters * 40  # many wide filters at once: items from several filters interleave
    got = e.messages_batch(filters)
    for f, g in zip(filters, got):
        assert g == o.messages(f), f


def test_messages_empty_topic_retained(gpu_available):
    """Q6: a retained packet on topic "" is returned for literal-final particles without a
    retain path (topics.go:573)."""
    e, o = EngineAdapter(), OracleAdapter()
    for ix in (e, o):
        ix.retain_message("", b"p", True, handle=99)
        ix.retain_message("a/b", b"p", True, handle=5)
        ix.subscribe("c", "a/c")
    for f in ["a/+", "+/c", "a/c", "+/+", "#", "a/b"]:
        assert e.messages(f) == o.messages(f), f


@pytest.mark.parametrize("image,spec_mb,edges", [(True, None, 1), (True, None, 0), (False, None, 1), (False, 0, 1),
                                                 (False, 3, 1)])
def test_messages_workload_parity(image, spec_mb, edges, gpu_available):
    """Messages on a config-5-shaped workload, over the level-order image (default) and the
    particle walk. spec_mb (walk): the speculative count's scratch budget (default: one walk for
    most filters; "0": count and fill walks; "3": a few hundred slots per filter, so that many
    filters overflow their scratch and are walked again)."""
    from mqmatch import workload as W
    from mqmatch import engine as E
    rb, ro, hd, rh = W.gen_retained(100000, n_sys=1000, seed=61)
    fb, fo = W.gen_msg_filters(rh, 5000, seed=62)
    eng, orc = E.Engine(), O.OracleIndex()
    if spec_mb is not None:
        eng.set_option(E.OPT_MSG_SPEC_MB, spec_mb)
    if not image:
        eng.set_option(E.OPT_MSG_IMAGE, 0)
    eng.set_option(E.OPT_MSG_EDGES, edges)  # (the image's edge table or the index's, image path)
    eng.retain_bulk(rb, ro, hd)
    orc.retain_bulk(rb, ro, hd)
    base, count, hs = eng.messages_batch(fb, fo)
    od, ocnt, _ = orc.messages_digest_batch(fb, fo)
    assert (count == ocnt).all()
    from digest import fold, SEED
    for i in range(len(count)):
        h = np.sort(hs[int(base[i]):int(base[i]) + int(count[i])])
        d = fold(SEED, np.uint64(len(h)))
        for x in h:
            d = fold(d, x)
        assert d == od[i], i


@pytest.mark.parametrize("keyidx", [1, 0])
def test_messages_key_index(keyidx, gpu_available):
    """Literal segments under wide runs (MQ_OPT_MSG_KEYIDX: the image's key index — one table
    probe, then per run wave-wide searches or a binary search per lane — or one edge-table probe
    per particle): short and long (hashed, byte-verified) keys, keys that no particle of the run
    has, keys some runs share, dense and sparse hits, one wide run (w/+/...) and some hundred runs
    (u/+/k/+/...), nested fan-outs; every filter equal to the oracle (topics.go:547-576)."""
    from mqmatch import engine as E
    e, o = E.Engine(), O.OracleIndex()
    e.set_option(E.OPT_MSG_KEYIDX, keyidx)
    longa, longb = "l" * 20 + "a", "l" * 20 + "b"
    topics, h = [], 0
    for i in range(200):
        for j in range(40):
            topics.append(f"u/{i}/k/{j}/{'m' if j % 3 else 'n'}")
        topics.append(f"u/{i}/j/0/m")
    for i in range(3000):
        topics.append(f"w/{i}/x")
        if i % 3 == 0:
            topics.append(f"w/{i}/{longa}")
        if i % 7 == 0:
            topics.append(f"w/{i}/{longb}/z")
        if i % 50 == 0:
            topics.append(f"v/{i}/x/q/{i % 4}")
        topics.append(f"v/{i}/y")
    for t in topics:
        h += 1
        assert e.retain_message(t, h, 1, True) == o.retain_message(t, h, 1, True)
    filters = ["w/+/x", f"w/+/{longa}", f"w/+/{longb}/+", f"w/+/{longb}/#", "w/+/nope", f"w/+/{'l' * 20}c",
               "+/+/x", "+/+/x/q/+", "+/+/x/+/1", "v/+/x/#", "+/+/y", "+/+/" + longa, "w/+/x/#", "+/+/+/q/#",
               "u/+/k/+/m", "u/+/k/+/n/#", "u/+/+/+/m", "+/+/k/+/n", "u/+/k/+/z"] * 8
    fb, fo = E.pack_strings(filters)
    base, count, hs = e.messages_batch(fb, fo)
    for i, f in enumerate(filters):
        got = sorted(hs[int(base[i]):int(base[i]) + int(count[i])].tolist())
        assert got == o.messages(f), f
    res = e.messages_runs_batch(fb, fo)
    assert _runs_sets(res, len(filters)) == [o.messages(f) for f in filters]
    e.close()


def _runs_sets(res, n):
    """Per-filter sorted handle lists of a Messages runs result (dict: run_base, n_runs, runs,
    handles), with each filter's runs checked to tile its [base, + count) of the expanded output."""
    out = []
    hs = res["handles"]
    for i in range(n):
        rb, nr = int(res["run_base"][i]), int(res["n_runs"][i])
        runs = res["runs"][rb:rb + nr]
        got = []
        at = sorted((int(r["at"]), int(r["count"])) for r in runs)
        pos = int(res["base"][i])
        for a, c in at:  # the runs tile the filter's part of the expanded output
            assert a == pos, (i, at)
            pos += c
        assert pos == int(res["base"][i]) + int(res["count"][i]), i
        for r in runs:
            got += hs[int(r["first"]):int(r["first"]) + int(r["count"])].tolist()
        out.append(sorted(got))
    return out


@pytest.mark.parametrize("q6", [False, True])
@pytest.mark.parametrize("seed", range(3))
def test_messages_runs_parity(seed, q6, gpu_available):
    """Messages as runs at the boundary (mq_messages_runs_batch / _device):
    each filter's runs index the retained image's handles (or, q6 — the "" entry live, the
    particle walk — the batch's own, one run per filter), tile its part of the expanded output,
    expand (mq_msg_runs_expand) to the handle result, and equal the oracle (topics.go:525-579)."""
    import torch
    from mqmatch import engine as E
    r = random.Random(3000 + seed)
    topics = ["/".join(r.choice(MSEGS) for _ in range(r.randint(1, 5))) for _ in range(400)]
    topics = [t for t in topics if t != ""] + ([""] if q6 else [])
    e, o = E.Engine(), O.OracleIndex()
    for i, t in enumerate(topics):
        pl = 0 if (r.random() < 0.1 and t != "") else 1
        ret = r.random() < 0.9
        assert e.retain_message(t, i + 1, pl, ret) == o.retain_message(t, i + 1, pl, ret), t
    for t in topics[::11]:
        if t:
            e.retained_delete(t)
            o.retained_delete(t)
    filters = ["/".join(r.choice(MSEGS + ["+", "+", "#"]) for _ in range(r.randint(1, 5))) for _ in range(300)]
    filters += ["#", "+", "+/+", "$SYS/#", "$SYS/+", "a/#", "a/+/#", "", "a", "a/b", "+/#", "+/+/#"]
    fb, fo = E.pack_strings(filters)
    n = len(filters)
    want = [o.messages(f) for f in filters]
    res = e.messages_runs_batch(fb, fo, expand=True)
    assert _runs_sets(res, n) == want
    for i in range(n):  # the expansion lays each filter out at its base
        b, c = int(res["base"][i]), int(res["count"][i])
        assert sorted(res["expanded"][b:b + c].tolist()) == want[i], filters[i]
    d_fb = torch.from_numpy(np.concatenate([fb, np.zeros(16, np.uint8)])).cuda()
    d_fo = torch.from_numpy(fo.view(np.int64)).cuda()
    torch.cuda.synchronize()
    dres = E.device_messages_runs(e.messages_runs_device(d_fb.data_ptr(), d_fo.data_ptr(), n), n)
    assert _runs_sets(dres, n) == want
    assert (dres["n_runs"] == 1).all() == q6  # (q6: the particle walk's one run per filter)
    e.close()


@pytest.mark.parametrize("export", [1, 0])
def test_messages_runs_workload(export, gpu_available):
    """Runs on a config-5-shaped workload (100k retained, 5k filters; wide fan-outs exported to
    work items or not): device and host runs digest-equal to the oracle, and far fewer runs than
    handles (the point of the format)."""
    import torch
    from mqmatch import workload as W
    from mqmatch import engine as E
    rb, ro, hd, rh = W.gen_retained(100000, n_sys=1000, seed=61)
    fb, fo = W.gen_msg_filters(rh, 5000, seed=62)
    n = len(fo) - 1
    eng, orc = E.Engine(), O.OracleIndex()
    eng.set_option(E.OPT_MSG_EXPORT, export)
    eng.retain_bulk(rb, ro, hd)
    orc.retain_bulk(rb, ro, hd)
    od, ocnt, _ = orc.messages_digest_batch(fb, fo)
    res = eng.messages_runs_batch(fb, fo)
    assert (res["count"] == ocnt).all()
    assert (O.run_digests(res) == od).all()
    d_fb = torch.from_numpy(np.concatenate([fb, np.zeros(16, np.uint8)])).cuda()
    d_fo = torch.from_numpy(fo.view(np.int64)).cuda()
    torch.cuda.synchronize()
    for _ in range(2):  # (the second batch on the buffers the first left: one synchronisation)
        dres = E.device_messages_runs(eng.messages_runs_device(d_fb.data_ptr(), d_fo.data_ptr(), n), n)
        assert (dres["count"] == ocnt).all()
        assert (O.run_digests(dres) == od).all()
    assert len(dres["runs"]) * 4 < int(ocnt.sum())
    base, count, hs = eng.messages_batch(fb, fo)  # the handle format after runs: unchanged
    assert (O.handle_digests(base, count, hs) == od).all()
    eng.close()


def test_messages_edge_table_tiers(gpu_available):
    """The retained image's edge table at each of its size tiers (device.cpp build_image: at most
    1/16 full within the budget, 1/8 within 4x the budget, else ~1/4 or denser). The product budget
    (8 GiB) is only exceeded at config 5's full size, so MQ_OPT_MSG_EDGE_BUDGET lowers it here until
    the table takes each sparser fallback; every tier's Messages equal the oracle's, and the table
    shrinks from tier to tier (topics.go:530-579)."""
    from mqmatch import workload as W
    from mqmatch import engine as E
    from digest import fold, SEED
    rb, ro, hd, rh = W.gen_retained(200000, n_sys=1000, seed=65)
    fb, fo = W.gen_msg_filters(rh, 6000, seed=66)
    orc = O.OracleIndex()
    orc.retain_bulk(rb, ro, hd)
    od, ocnt, _ = orc.messages_digest_batch(fb, fo)

    def run(budget_mb):
        eng = E.Engine()
        if budget_mb is not None:
            eng.set_option(E.OPT_MSG_EDGE_BUDGET, budget_mb)
        eng.retain_bulk(rb, ro, hd)
        eng.profile(True)
        base, count, hs = eng.messages_batch(fb, fo)
        p = eng.profile_read()
        assert (count == ocnt).all(), budget_mb
        dg = O.handle_digests(base, count, hs)
        assert (dg == od).all(), budget_mb
        return p["msg_edge_slots"][0], p["msg_edge_particles"][0]

    slots16, lo = run(None)
    assert slots16 >= 16 * lo
    full_mb = slots16 * 32 >> 20  # (32 B per slot)
    slots8, _ = run(full_mb // 2)  # over the 1/16 budget, within 4x of it: the 1/8 tier
    assert slots8 == slots16 // 2 and slots8 < 16 * lo
    slots4, _ = run(max(1, full_mb // 16))  # over 4x the budget too: ~1/4
    assert slots4 <= slots8 // 2 and slots4 >= 2 * lo
    slots_min, _ = run(1)  # the densest table the loop allows (load < 1/2)
    assert slots_min <= slots4 and slots_min > 2 * lo


def _submit(eng, tb, to):
    import ctypes as C
    from mqmatch import engine as E
    t = C.c_void_p()
    rc = E.lib().mq_match_spans_submit(eng.h, E._p(tb, E._u8p), E._p(to, E._u64p), len(to) - 1, C.byref(t))
    return rc, t


def _wait(t, n):
    import ctypes as C
    from mqmatch import engine as E
    rp = C.POINTER(E.SpanResult)()
    rc = E.lib().mq_match_spans_wait(t, C.byref(rp))
    return rc, (E._expand_host_spans(rp, n) if rc == 0 else None)


@pytest.mark.parametrize("inline", [True, False])
def test_pipelined_submit_fails_then_recovers(inline, gpu_available):
    """A pipelined submit whose batch fails (MQ_OPT_FAIL_NEXT: as if a kernel guard tripped) returns
    MQ_EIO and arms no copy into the freed result: the batch submitted before it still waits to its
    exact result, and later submits and waits are exact. inline=True: an index with an inline
    subscription (batches are not one-sync: the error is read at the batch's end, after its result
    was packed); False: one-sync batches (a copy armed before the error check)."""
    from mqmatch import engine as E
    from mqmatch import workload as W
    w, eng, orc = _workload_pair(40000, 3000, seed=91)
    if inline:  # (on "#", every topic gathers it; its filter id is the workload's: ids name filter strings)
        offs = w["offs"].astype(np.int64)
        fid = next(int(w["filter_ids"][i]) for i in range(len(offs) - 1) if bytes(w["bytes"][offs[i]:offs[i + 1]]) == b"#")
        assert eng.inline_subscribe("#", 7, fid) == bool(orc.inline_subscribe("#", 7, filter_id=fid))
    batches = [W.gen_topics(w, 3000, seed=92 + i) for i in range(4)]
    want = [orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))[0] for tb, to in batches]
    rc, t0 = _submit(eng, *batches[0])
    assert rc == 0
    eng.set_option(E.OPT_FAIL_NEXT, 1)
    rc, t1 = _submit(eng, *batches[1])
    assert rc == E.MQ_EIO and not t1
    rc, r0 = _wait(t0, 3000)  # (its copy was issued by the failed submit's flush)
    assert rc == 0 and (engine_digests(r0)[0] == want[0]).all()
    rc, t2 = _submit(eng, *batches[2])
    assert rc == 0
    rc, t3 = _submit(eng, *batches[3])
    assert rc == 0
    for t, k in ((t2, 2), (t3, 3)):
        rc, r = _wait(t, 3000)
        assert rc == 0 and (engine_digests(r)[0] == want[k]).all(), k
    # a failure with no batch before it, then a plain host match
    eng.set_option(E.OPT_FAIL_NEXT, 1)
    rc, _ = _submit(eng, *batches[1])
    assert rc == E.MQ_EIO
    _digest_parity(eng, orc, *batches[1], fmts=("spans",))


@pytest.mark.parametrize("fmt", FORMATS)
def test_gather_slot_overflow(fmt, gpu_available):
    """A topic matching > 64 particles overflows its count-pass gather slots and takes the
    compact fill pass; mixed with ordinary topics in one batch."""
    e, o = EngineAdapter(fmt), OracleAdapter()
    levels = [f"l{i}" for i in range(50)]
    for d in range(1, 50):
        f = "/".join(levels[:d]) + "/#"
        for c in (f"c{d % 7}", "cz"):
            assert e.subscribe(c, f, identifier=d) == o.subscribe(c, f, identifier=d)
        e.inline_subscribe(f, d % 5)
        o.inline_subscribe(f, d % 5)
    e.subscribe("cq", "l0/+/l2")
    o.subscribe("cq", "l0/+/l2")
    topics = ["/".join(levels[:k]) for k in (1, 3, 10, 33, 34, 40, 50)] + ["l0/x/l2", "q"]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


@pytest.mark.parametrize("fmt", FORMATS)
def test_many_merging_clients(fmt, gpu_available):
    """600 clients each with three co-matching filters in one topic (bases, max Qos, ident rows),
    next to clients whose partners are not gathered for the topic (plain rows)."""
    e, o = EngineAdapter(fmt), OracleAdapter()
    for i in range(600):
        c = f"m{i}"
        for f, ident in (("o/#", i % 3), ("o/p", 1 + i % 5), ("o/+", 0)):
            assert e.subscribe(c, f, identifier=ident, qos=i % 3) == o.subscribe(c, f, identifier=ident, qos=i % 3)
    for i in range(100):  # partners that are not gathered for "o/p": emitted directly
        e.subscribe(f"s{i}", "o/q")
        o.subscribe(f"s{i}", "o/q")
        e.subscribe(f"s{i}", "o/#")
        o.subscribe(f"s{i}", "o/#")
    topics = ["o/p", "o/q", "o", "o/z", "o/p/x"]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


@pytest.mark.parametrize("exp", [0, 512])
def test_set_pass_big_gathers(exp, gpu_available):
    """Merge gathers far beyond the set pass's hash fold: 5,000 clients on "o/#" (more may-merge
    records than one pass of the bit fold holds, kBitRecs = 2048) with partners at "o/p", "o/+",
    "+/p" and "o/p/#" (Qos 0-2, NoLocal, identifiers 0-4), next to clients with one filter; topics
    that gather every subset of them. Device and host span results equal the oracle's (exp 512: the
    partner-link path the bit fold replaced)."""
    import random as R
    import torch
    from mqmatch import engine as E
    rng = R.Random(97)
    e, o = EngineAdapter("spans"), OracleAdapter()
    e.x.engine.set_option(E.OPT_SET_EXP, exp)
    for i in range(5000):
        c = f"m{i}"
        for f in ("o/#", "o/p", "o/+", "+/p", "o/p/#"):
            if f != "o/#" and rng.random() < 0.35:
                continue
            q, ident, nl = rng.randrange(3), rng.randrange(5), rng.random() < 0.2
            assert e.subscribe(c, f, qos=q, identifier=ident, no_local=nl) == o.subscribe(c, f, qos=q, identifier=ident,
                                                                                        no_local=nl)
    for i in range(500):
        assert e.subscribe(f"s{i}", "o/#") == o.subscribe(f"s{i}", "o/#")
    topics = ["o/p", "o/q", "o", "x/p", "o/p/x", "o/p/x/y"] * 20
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t
    # device results of a batch large enough for the one-sync path (merge sets formed over it)
    from mqmatch import workload as W
    raw, offs = E.pack_strings(topics * 600)
    n = len(offs) - 1
    d_tb = torch.from_numpy(np.concatenate([raw, np.zeros(16, np.uint8)])).cuda()
    d_to = torch.from_numpy(offs.view(np.int64)).cuda()
    torch.cuda.synchronize()
    # (digests name clients and filters by the adapter's ids: compare through the same adapter)
    want = {t: o.subscribers(t) for t in set(topics)}
    r = e.x.engine.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)
    res = E.expand_device_spans(r, n)
    got = e.x._rebuild(res, 0)  # (first topic through the mirror's rematerialisation)
    assert canonical(got) == want[topics[0]]
    for i in range(0, n, 997):
        assert canonical(e.x._rebuild(res, i)) == want[(topics * 600)[i]], i


@pytest.mark.parametrize("fmt", FORMATS)
def test_partner_map_fallback(fmt, gpu_available):
    """Topics gathering 128 (the pair analysis' limit), 256 and 512 (linear partner lookup)
    nodes that all hold may-merge subscriptions: every literal/'+' path of depth 7, 8 and 9."""
    import itertools
    e, o = EngineAdapter(fmt), OracleAdapter()
    for depth in (7, 8, 9):
        paths = ["/".join(f"a{i}" if b == 0 else "+" for i, b in enumerate(bits))
                 for bits in itertools.product((0, 1), repeat=depth)]
        for k, f in enumerate(paths):  # client k holds paths k and k + 1: partners pairwise
            for g in (f, paths[(k + 1) % len(paths)]):
                c = f"d{depth}c{k}"
                kw = dict(qos=(k + len(g)) % 3, identifier=(k % 4) * 7, no_local=k % 5 == 0)
                assert e.subscribe(c, g, **kw) == o.subscribe(c, g, **kw)
    topics = ["/".join(f"a{i}" for i in range(9)), "/".join(f"a{i}" for i in range(8)),
              "/".join(f"a{i}" for i in range(7)), "/".join(f"a{i}" for i in range(8)) + "/x", "a0/a1"]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


@pytest.mark.parametrize("fmt", FORMATS)
def test_many_pair_hits(fmt, gpu_available):
    """A topic whose merge gathers are pairwise partners through many clients: hundreds of
    (g, h) hit lists, staged and resolved in several flushes (span format: more lists than LDS
    holds, so the pair analysis counts first, reserves the patches, then resolves)."""
    e, o = EngineAdapter(fmt), OracleAdapter()
    r = random.Random(77)
    fs = ["#", "a/#", "+/#", "a/b/#", "a/+/#", "+/b/#", "+/+/#", "a/b/c/#", "a/b/+/#", "+/b/c/#",
          "a/+/c/#", "+/+/c/#", "a/b/c/d", "a/b/c/+", "a/+/c/d", "+/b/c/d", "+/+/+/+", "a/b/+/d",
          "+/+/c/d", "a/+/+/d", "a/b/c/d/#"]
    for c in range(40):
        mine = fs if c < 3 else r.sample(fs, r.randint(2, 8))
        for f in mine:
            kw = dict(qos=r.randint(0, 2), identifier=r.choice([0, 0, 4, 11]), no_local=r.random() < 0.3)
            assert e.subscribe(f"p{c}", f, **kw) == o.subscribe(f"p{c}", f, **kw)
    topics = ["a/b/c/d", "a/b/c", "a/x/c/d", "$SYS/b/c/d", "a/b/c/d/e", "q"]
    for t, g in zip(topics, e.subscribers_batch(topics)):
        assert g == o.subscribers(t), t


def test_cpp_host_mirror(gpu_available):
    """The reference's topics_test.go cases restated in C++ against the C++ host mirror of the
    Go API (mqtt-server_amd/csrc/host), running on the GPU engine."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "mqtt-server_amd", "build", "test_topics_index")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_acl_match_topic_batch(gpu_available):
    """Batched auth.MatchTopic (hooks/auth/ledger.go:90-118) on the GPU: the reference's own cases
    (ledger_test.go:461-493) and random filter/topic pairs, against the oracle's restatement."""
    from mqmatch import engine as E
    eng = E.Engine()
    kat = [("a/+/c/+", "a/b/c/d"), ("a/+/+/+", "a/b/c/d"), ("stuff/#", "stuff/things/yeah"),
           ("a/+/#/+", "a/b/c/d/as/dds"), ("test", "test"), ("things/stuff//", "things/stuff/"), ("t", "t2"),
           (" ", "  ")]
    r = random.Random(71)
    segs = ["a", "b", "c", "", "+", "#", "longersegment-abcdefgh", "ü"]
    filters = [k[0] for k in kat] + ["/".join(r.choice(segs) for _ in range(r.randint(1, 5))) for _ in range(300)]
    topics = [k[1] for k in kat] + ["/".join(r.choice(segs[:4] + segs[6:]) for _ in range(r.randint(1, 6)))
                                    for _ in range(200)] + [""]
    pf = list(range(len(kat))) + [r.randrange(len(filters)) for _ in range(20000)]
    pt = list(range(len(kat))) + [r.randrange(len(topics)) for _ in range(20000)]
    got = eng.acl_match_batch(filters, topics, pf, pt)
    for f, t, g in zip(pf, pt, got):
        assert g == O.match_topic(filters[f], topics[t]), (filters[f], topics[t])
    assert sum(m for _, m in got) > 1000
