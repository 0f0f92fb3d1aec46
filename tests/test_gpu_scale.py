"""Parity at the benchmark's own scale: the headline configuration
(10M subscriptions, config-3 mix, SURVEY.md §8d generator) and the IoT fan-in mix at 5M
subscriptions, through the C-ABI in both result formats, digest-equal to the oracle on a
4096-topic (IoT: 20000-topic) sample of the bench's own batch. Besides the sample, every topic
of a 1M-topic batch is checked for size-independent properties of the span format (counts add
up, patches in range, no patches where no client has two matches)."""
import os

import numpy as np
import pytest

import oracle as O
from digest import engine_digests

pytestmark = pytest.mark.gpu


def _parity(eng, orc, tb, to, fmts=("spans", "rows")):
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
    for fmt in fmts:
        res = eng.match_batch_spans(tb, to) if fmt == "spans" else eng.match_batch(tb, to)
        dg, cnt = engine_digests(res)
        bad = np.nonzero(dg != od)[0]
        assert len(bad) == 0, f"{fmt}: {len(bad)} of {len(dg)} topics differ, first {bad[:5]}"
        assert (cnt == ocnt).all()
    return ocnt


def test_headline_10m_subscriptions(gpu_available):
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(10_000_000, 1_000_000, seed=W.BASE_SEED)  # bench.py's index
    eng = E.Engine(expected_subs=10_000_000)
    new = eng.subscribe_bulk(w)
    orc = O.OracleIndex()
    assert (orc.subscribe_bulk(w) == new).all()
    tb, to = W.gen_topics(w, 1_000_000, seed=W.BASE_SEED)  # bench.py's rank-0 batch
    cnt = _parity(eng, orc, tb, to[:4097])
    assert cnt[:, 0].mean() > 1000  # the workload really fans out
    del orc
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


def test_iot_5m_subscriptions(gpu_available):
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(5_000_000, 5_000_000, seed=W.BASE_SEED, mix=W.MIX_IOT)
    eng = E.Engine(expected_subs=5_000_000)
    new = eng.subscribe_bulk(w)
    orc = O.OracleIndex()
    assert (orc.subscribe_bulk(w) == new).all()
    tb, to = W.gen_topics(w, 20000, seed=W.BASE_SEED, mix=W.MIX_IOT)
    _parity(eng, orc, tb, to)
