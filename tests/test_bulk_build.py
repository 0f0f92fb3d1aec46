"""The bulk restore path (mq_subscribe_bulk / mq_retain_bulk on an empty index,
csrc/engine/index_bulk.cpp; server.go:1624-1640 loadSubscriptions, server.go:1688-1692
loadRetained) builds the image the per-entry path builds: the same answers (out_new), the
same live counts (mq_index_stats), the same invariants (mq_index_check), an image that takes
later updates — and, on the GPU, the same match results (digests) for Subscribers and
Messages. The per-entry image is built by the same calls on a non-empty index (one entry
first), which the bulk path hands to the per-entry loop."""
import random

import numpy as np
import pytest

from mqmatch import engine as E
from mqmatch import workload as W
from digest import engine_digests

SEGS = ["a", "b", "c", "", "+", "#", "$SYS", "$share", "$SHARE", "g", "x", "dev", "longersegment-abcdefghijk"]


def _entries(seed, n, n_clients=300):
    r = random.Random(seed)
    out = []
    for _ in range(n):
        f = "/".join(r.choice(SEGS) for _ in range(r.randint(1, 6)))
        if r.random() < 0.1:
            f = "$share/g%d/" % r.randrange(4) + f
        out.append((f, r.randrange(n_clients), r.randint(0, 2), r.choice([0, 0, 1, 2, 5, 8]), r.choice([0, 0, 3, 9])))
    return out


def _pack(ents):
    fids = {}
    bs = [e[0].encode() for e in ents]
    offs = np.zeros(len(bs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    return {"bytes": np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy(), "offs": offs,
            "client_ids": np.array([e[1] for e in ents], np.uint32),
            "filter_ids": np.array([fids.setdefault(e[0], len(fids)) for e in ents], np.uint32),
            "qos": np.array([e[2] for e in ents], np.uint8), "flags": np.array([e[3] for e in ents], np.uint8),
            "idents": np.array([e[4] for e in ents], np.int32)}


def _slice(w, lo, hi):
    o = w["offs"][lo:hi + 1]
    return {"bytes": w["bytes"][int(o[0]):int(o[-1])].copy() if int(o[-1]) > int(o[0]) else np.zeros(1, np.uint8),
            "offs": (o - o[0]).astype(np.uint64),
            **{k: w[k][lo:hi] for k in ("client_ids", "filter_ids", "qos", "flags", "idents")}}


def _pair(w, **kw):
    """(bulk engine, out_new), (per-entry engine, out_new) over the same entries."""
    n = len(w["client_ids"])
    a = E.Engine(**kw)
    oa = a.subscribe_bulk(w)
    b = E.Engine(**kw)
    ob = np.concatenate([b.subscribe_bulk(_slice(w, 0, 1)), b.subscribe_bulk(_slice(w, 1, n))])
    return (a, oa), (b, ob)


@pytest.mark.parametrize("n_shards", [1, 2, 3])
def test_bulk_subscribe_equals_per_entry(n_shards):
    w = _pack(_entries(11 + n_shards, 9000))
    for k in range(n_shards):
        (a, oa), (b, ob) = _pair(w, shard=k, n_shards=n_shards)
        assert (oa[:len(w["client_ids"])] == ob[:len(w["client_ids"])]).all()
        assert a.stats() == b.stats()
        a.check()
        b.check()


def test_bulk_image_takes_updates():
    ents = _entries(5, 8000)
    w = _pack(ents)
    (a, _), (b, _) = _pair(w)
    r = random.Random(9)
    for step in range(3000):
        f, c, q, fl, i = r.choice(ents) if r.random() < 0.7 else _entries(100 + step, 1)[0]
        if r.random() < 0.5:
            assert a.unsubscribe(f, c) == b.unsubscribe(f, c)
        else:
            fid = 10_000 + step
            assert a.subscribe(f, c, fid, q, fl, i) == b.subscribe(f, c, fid, q, fl, i)
    assert a.stats() == b.stats()
    a.check()
    b.check()


def test_bulk_unsubscribe_equals_per_entry():
    """mq_unsubscribe_bulk answers exactly as mq_unsubscribe, in order (repeats, unknown clients,
    filters never subscribed), and leaves the same image."""
    ents = _entries(21, 6000)
    w = _pack(ents)
    (a, _), (b, _) = _pair(w)
    r = random.Random(22)
    pairs = [(f, c) for f, c, _, _, _ in r.sample(ents, 2500)] + [("no/such/filter", 1), (ents[3][0], 999)]
    pairs += pairs[:100]  # (already removed: false, the particle may be gone)
    bs = [f.encode() for f, _ in pairs]
    offs = np.zeros(len(bs) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in bs])
    got = a.unsubscribe_bulk(np.frombuffer(b"".join(bs), np.uint8).copy(), offs,
                             np.array([c for _, c in pairs], np.uint32))
    want = [b.unsubscribe(f, c) for f, c in pairs]
    assert got.tolist() == want
    assert a.stats() == b.stats()
    a.check()
    b.check()


def _retained(seed, n):
    r = random.Random(seed)
    ts = ["/".join(r.choice(["a", "b", "c", "", "x", "$SYS", "dev"]) for _ in range(r.randint(1, 6)))
          for _ in range(n)]
    ts[7] = ""  # the Retained entry without a retain path
    bs = [t.encode() for t in ts]
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    return np.frombuffer(b"".join(bs), np.uint8).copy(), offs, np.arange(1, n + 1, dtype=np.uint64) * 7


@pytest.mark.parametrize("n_shards", [1, 2])
def test_bulk_retain_equals_per_entry(n_shards):
    rb, ro, hd = _retained(3, 9000)
    for k in range(n_shards):
        a, b = E.Engine(shard=k, n_shards=n_shards), E.Engine(shard=k, n_shards=n_shards)
        a.retain_bulk(rb, ro, hd)
        b.retain_bulk(rb, ro[:2] - ro[0], hd[:1])
        b.retain_bulk(rb[int(ro[1]):], (ro[1:] - ro[1]).astype(np.uint64), hd[1:])
        assert a.retained_len() == b.retained_len()
        assert a.stats() == b.stats()
        a.check()
        b.check()


@pytest.mark.gpu
def test_bulk_images_match_identically(gpu_available):
    """Subscribers and Messages over the bulk image equal those over the per-entry image."""
    w = W.gen_subscriptions(200_000, 20_000)
    (a, _), (b, _) = _pair(w)
    tb, to = W.gen_topics(w, 20_000)
    da, ca = engine_digests(a.match_batch(tb, to))
    db, cb = engine_digests(b.match_batch(tb, to))
    assert (ca == cb).all() and (da == db).all()
    rb, ro, hd, rh = W.gen_retained(100_000, n_sys=500)
    a, b = E.Engine(), E.Engine()  # empty images: the bulk path and the per-entry loop
    a.retain_bulk(rb, ro, hd)
    b.retain_bulk(rb, ro[:2] - ro[0], hd[:1])
    b.retain_bulk(rb[int(ro[1]):], (ro[1:] - ro[1]).astype(np.uint64), hd[1:])
    fb, fo = W.gen_msg_filters(rh, 5_000)
    ba, na, ha = a.messages_batch(fb, fo)
    bb, nb, hb = b.messages_batch(fb, fo)
    assert (na == nb).all()
    for i in range(len(na)):
        assert set(ha[ba[i]:ba[i] + na[i]].tolist()) == set(hb[bb[i]:bb[i] + nb[i]].tolist())


@pytest.mark.gpu
def test_churn_after_sync_matches_oracle(gpu_available):
    """Incremental sync (Device::sync: dirty 512-byte pages of every mirror, packed into one
    staging upload and scattered on the device): a bulk-built, synced index takes rounds of
    Unsubscribe / Subscribe churn, and each round's matches equal the oracle's."""
    import oracle as O
    from digest import engine_digests
    w = W.gen_subscriptions(200_000, 20_000)
    e, o = E.Engine(), O.OracleIndex()
    e.subscribe_bulk(w)
    o.subscribe_bulk(w)
    tb, to = W.gen_topics(w, 4096)
    raw, offs = w["bytes"].tobytes(), w["offs"]
    rng = np.random.default_rng(3)
    nxt = int(w["client_ids"].max()) + 1
    n = len(w["client_ids"])
    for rnd in range(4):
        dg, cnt = engine_digests(e.match_batch_spans(tb, to))
        od, ocnt, _ = o.digest_batch(tb, to)
        assert (dg == od).all() and (cnt == ocnt).all(), rnd
        up0 = e.stats()["upload_bytes_total"]
        for i in rng.choice(n, 500 * (rnd + 1), replace=False):
            f = raw[int(offs[i]):int(offs[i + 1])].decode("utf-8", "surrogateescape")
            c = int(w["client_ids"][i])
            assert e.unsubscribe(f, c) == o.unsubscribe(f, "c%07d" % c)
            q, fl, ident = int(w["qos"][i]), int(w["flags"][i]), int(w["idents"][i])
            assert e.subscribe(f, nxt, int(w["filter_ids"][i]), q, fl, ident) == \
                o.subscribe("c%07d" % nxt, f, q, ident, bool(fl & 1), bool(fl & 2), (fl >> 2) & 3,
                            client_id=nxt, filter_id=int(w["filter_ids"][i]))
            nxt += 1
        e.sync()
        assert e.stats()["upload_bytes_total"] - up0 < 64 * 1024 * 500 * (rnd + 1)  # pages, not arrays
