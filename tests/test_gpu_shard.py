"""Sharded matching (north star) against the oracle: G shard
indices (one handle each, all on GPU 0 here), every update issued to every shard, every shard
matching the full batch (mq_match_spans_begin), the exported cross-shard lists exchanged, and
each shard resolving its records (mq_match_spans_end). The shards' results are disjoint, so
their per-category digest parts add up to the single index's digest — compared with the
oracle's, bit for bit."""
import os
import random

import numpy as np
import pytest

import oracle as O
from digest import engine_digest_parts, fold_parts

pytestmark = pytest.mark.gpu


def _sharded_digests(shards, tb, to, device=False):
    """device=False: host results (mq_match_spans_end_host, per-topic patches); True: device
    results (mq_match_spans_end, merge sets' patches referenced and translated as a device
    consumer would)."""
    import torch
    from mqmatch import engine as E
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    xs = [e.match_spans_begin(d_tb.data_ptr(), d_to.data_ptr(), n) for e in shards]
    counts = np.zeros((n, 4), np.int64)
    sums = np.zeros((n, 4), np.uint64)
    for k, e in enumerate(shards):
        foreign = [x for j, x in enumerate(xs) if j != k]
        if device:
            res = E.expand_device_spans(e.match_spans_end(foreign), n)
        else:
            res = e.match_spans_end_expanded(foreign, n)
        c, s = engine_digest_parts(res)
        counts += c
        with np.errstate(over="ignore"):
            sums += s
    return fold_parts(counts, sums), counts, sum(int(x.n_ents) for x in xs)


def _build(n_shards, w, extra):
    from mqmatch import engine as E
    shards = [E.Engine(shard=k, n_shards=n_shards) for k in range(n_shards)]
    orc = O.OracleIndex()
    ref = orc.subscribe_bulk(w)
    for e in shards:
        got = e.subscribe_bulk(w)
        assert (got <= ref).all()
    for c, f, q, ident in extra:
        for e in shards:
            e.subscribe(f, c, 10_000_000 + hash(f) % 1_000_000, q, 0, ident)
        orc.subscribe(f"c{c:07d}", f, q, ident, client_id=c, filter_id=10_000_000 + hash(f) % 1_000_000)
    return shards, orc


@pytest.mark.parametrize("n_shards,device", [(2, False), (3, False), (3, True)])
def test_sharded_workload_parity(n_shards, device, gpu_available):
    from mqmatch import workload as W
    w = W.gen_subscriptions(120000, 6000, seed=81)
    shards, orc = _build(n_shards, w, [])
    tb, to = W.gen_topics(w, 6000, seed=82)
    dg, cnt, n_ents = _sharded_digests(shards, tb, to, device=device)
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
    assert (cnt == ocnt).all()
    bad = np.nonzero(dg != od)[0]
    assert len(bad) == 0, f"{len(bad)} topics differ, first {bad[:5]}"
    assert n_ents > 0 and cnt[:, 1].sum() > 0  # cross-shard nodes exported; identifier rows exist
    for e in shards:
        e.check()


@pytest.mark.parametrize("one_sync,patch_cap", [(1, 0), (1, 64), (0, 0)])
def test_sharded_begin_end_sync_modes(one_sync, patch_cap, gpu_available):
    """The sharded step's synchronisation modes, three batches each (the first one-sync begin finds
    no buffers from earlier batches and runs again host-sized; the later ones fit): the one-sync
    begin (export from k_desc, packed by k_xpack; walk-fused) and end; with 64-slot patch pools
    (the one-sync end overflows and runs again host-sized, the begin's results and the imported
    lists kept); MQ_OPT_ONE_SYNC 0 (the classic begin, k_xlist). Device and host results equal the
    oracle every batch."""
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(150000, 8000, seed=85)
    shards, orc = _build(4, w, [])
    for e in shards:
        e.set_option(E.OPT_ONE_SYNC, one_sync)
        if patch_cap:
            e.set_option(E.OPT_PATCH_CAP, patch_cap)
    for b, k in enumerate((3000, 9000, 9000)):
        tb, to = W.gen_topics(w, k, seed=86 + b)
        od, ocnt, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
        for device in (True, False):
            dg, cnt, n_ents = _sharded_digests(shards, tb, to, device=device)
            assert (cnt == ocnt).all(), (b, device)
            bad = np.nonzero(dg != od)[0]
            assert len(bad) == 0, f"batch {b} device={device}: {len(bad)} topics differ, first {bad[:5]}"
            assert n_ents > 0


@pytest.mark.parametrize("device", [False, True])
def test_config3_eight_shards(device, gpu_available):
    """Config 3 in its stated form on one GPU: the config-3 mix at 1M
    subscriptions sharded by filter hash over 8 shard handles, every shard matching the full
    4096-topic batch, the exported cross-shard lists exchanged, merge-set dedup on every shard
    (sets keyed by the local merge gathers and the other shards' entries). The shards' disjoint
    results add up to the oracle's digests, bit for bit, with host and device results."""
    from mqmatch import workload as W
    w = W.gen_subscriptions(1_000_000, 100_000, seed=W.BASE_SEED)
    shards, orc = _build(8, w, [])
    tb, to = W.gen_topics(w, 4096, seed=W.BASE_SEED)
    dg, cnt, n_ents = _sharded_digests(shards, tb, to, device=device)
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=min(16, os.cpu_count() or 8))
    assert (cnt == ocnt).all()
    bad = np.nonzero(dg != od)[0]
    assert len(bad) == 0, f"{len(bad)} topics differ, first {bad[:5]}"
    assert n_ents > 0 and cnt[:, 1].sum() > 0


@pytest.mark.parametrize("device", [False, True])
def test_sharded_many_merging_clients(device, gpu_available):
    """Clients whose co-matching filters are spread over the shards: bases, max Qos, OR'd NoLocal
    and identifier rows decided across shards (the rank keys order them)."""
    from mqmatch import engine as E
    n_shards = 3
    shards = [E.Engine(shard=k, n_shards=n_shards) for k in range(n_shards)]
    o = O.OracleIndex()
    r = random.Random(83)
    fs = ["#", "a/#", "+/#", "a/b/#", "a/+/#", "+/b/#", "+/+/#", "a/b/c/#", "a/b/+/#", "+/b/c/#", "a/+/c/#",
          "a/b/c/d", "a/b/c/+", "a/+/c/d", "+/b/c/d", "+/+/+/+", "a/b/+/d", "+/+/c/d", "a/+/+/d", "a/b/c/d/#"]
    fid = {f: i for i, f in enumerate(fs)}
    for c in range(300):
        for f in r.sample(fs, r.randint(1, 7)):
            q, ident, nl = r.randint(0, 2), r.choice([0, 0, 4, 11]), r.random() < 0.3
            for e in shards:
                e.subscribe(f, c, fid[f], q, 1 if nl else 0, ident)
            o.subscribe(f"c{c}", f, q, ident, nl, client_id=c, filter_id=fid[f])
    topics = ["a/b/c/d", "a/b/c", "a/x/c/d", "$SYS/b/c/d", "a/b/c/d/e", "q", "a", "x/b/c/d"]
    tb, to = E.pack_strings(topics)
    dg, cnt, _ = _sharded_digests(shards, tb, to, device=device)
    od, ocnt, _ = o.digest_batch(tb, to, nthreads=4)
    assert (cnt == ocnt).all() and (dg == od).all()


@pytest.mark.parametrize("device", [False, True])
def test_sharded_deep_ties_match_oracle(device, gpu_available):
    """Filters of one client on different shards agreeing in their first 32 levels' kinds (the
    rank keys tie): the deep-path codes order them (layout.h DeepTail, merge.hip deep_before) —
    deeper '+' / '#' / literal levels, a 32-level filter that is a proper prefix of a deeper one,
    and paths beyond 48 levels (a second code word). The shards' results equal the oracle's."""
    from mqmatch import engine as E
    n_shards = 3
    shards = [E.Engine(shard=k, n_shards=n_shards) for k in range(n_shards)]
    o = O.OracleIndex()
    pre = "/".join(f"l{i}" for i in range(32))
    pre52 = pre + "/" + "/".join(f"m{i}" for i in range(20))
    fs = [pre, pre + "/#", pre + "/x", pre + "/+", pre + "/x/#", pre + "/x/y", pre + "/x/+", pre + "/+/y",
          pre + "/+/#", pre + "/+/+", "/".join(["+"] * 32) + "/x/y", pre52, pre52 + "/#", pre52 + "/z",
          pre52 + "/+", pre52 + "/z/#", pre + "/m0/#"]
    owners = set()
    r = random.Random(87)
    for c in range(60):
        for f in r.sample(fs, r.randint(2, 8)):
            q, ident, nl = r.randint(0, 2), r.choice([0, 3, 9]), r.random() < 0.3
            for k, e in enumerate(shards):
                if e.subscribe(f, c, fs.index(f), q, 1 if nl else 0, ident) == 1:
                    owners.add(k)
            o.subscribe(f"c{c}", f, q, ident, nl, client_id=c, filter_id=fs.index(f))
    assert len(owners) >= 2, owners
    topics = [pre, pre + "/x", pre + "/x/y", pre + "/q/y", pre + "/x/q", pre52, pre52 + "/z", pre52 + "/z/w",
              pre + "/m0", "/".join(f"l{i}" for i in range(31))]
    tb, to = E.pack_strings(topics)
    dg, cnt, n_ents = _sharded_digests(shards, tb, to, device=device)
    od, ocnt, _ = o.digest_batch(tb, to, nthreads=4)
    assert n_ents > 0
    assert (cnt == ocnt).all()
    bad = np.nonzero(dg != od)[0]
    assert len(bad) == 0, f"topics {[topics[i] for i in bad]} differ"
    for e in shards:
        e.check()


@pytest.mark.parametrize("device", [False, True])
def test_sharded_deep_filter_id_reuse(device, gpu_available):
    """A filter id that named a deep filter (beyond 32 levels: a DeepTail entry, layout.h) is reused
    for a 32-level filter once the deep one is gone from every shard: the entry went
    with its last holder (Index::deep_unref), so the 32-level filter's tie with a deeper filter on
    another shard is ordered as its proper prefix — first — and the merged
    rows equal the oracle's."""
    from mqmatch import engine as E
    shards = [E.Engine(shard=k, n_shards=2) for k in range(2)]
    o = O.OracleIndex()

    def sub(c, f, fid, q, nl=False, ident=0):
        own = [e.subscribe(f, c, fid, q, 1 if nl else 0, ident) for e in shards]
        o.subscribe(f"c{c}", f, q, ident, nl, client_id=c, filter_id=fid)
        return own

    def unsub(c, f):
        for e in shards:
            e.unsubscribe(f, c)
        o.unsubscribe(f, f"c{c}")

    def owner(f):
        own = [e.subscribe(f, 999, 77, 0, 0, 0) for e in shards]
        for e in shards:
            e.unsubscribe(f, 999)
        return own.index(1)

    for j in range(64):  # a 32-level prefix whose filter and its '#' child live on different shards
        pre = "/".join(f"p{j}x{i}" for i in range(32))
        if owner(pre) != owner(pre + "/#"):
            break
    else:
        pytest.fail("no prefix splits over the shards")
    topics = [pre, pre + "/x", pre + "/x/y"]
    tb, to = E.pack_strings(topics)
    # fid 5 names the deep filter pre/#, which reaches the device, then leaves every shard
    for c in range(12):
        sub(c, pre + "/#", 5, c % 3)
        sub(c, pre + "/x/+", 8, (c + 1) % 3)
    _sharded_digests(shards, tb, to, device=device)
    for c in range(12):
        unsub(c, pre + "/#")
    # fid 5 reused for the 32-level pre; pre/# back under fid 6
    for c in range(12):
        sub(c, pre, 5, c % 3, nl=c % 4 == 0, ident=c % 5)
        sub(c, pre + "/#", 6, (c + 2) % 3, ident=(c + 1) % 4)
    dg, cnt, n_ents = _sharded_digests(shards, tb, to, device=device)
    od, ocnt, _ = o.digest_batch(tb, to, nthreads=2)
    assert n_ents > 0
    assert (cnt == ocnt).all()
    bad = np.nonzero(dg != od)[0]
    assert len(bad) == 0, f"topics {[topics[i] for i in bad]} differ"
    for e in shards:
        e.check()
