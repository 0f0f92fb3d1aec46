"""CPU tests of the engine library: it loads, exports every symbol include/mqmatch.h declares,
and its host-side update logic (Subscribe/Unsubscribe/Inline*/RetainMessage return values,
trie shape after trims) equals the oracle on random operation sequences. No GPU is touched:
the device image is created lazily by the first sync/match."""
import os
import random
import re

import pytest

from mqmatch import engine as E
import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(REPO, "include", "mqmatch.h")).read()
    inline = set(re.findall(r"static inline \w+ (mq_[a-z_]+)\s*\(", hdr))  # header-only helpers
    return sorted(set(re.findall(r"\b(mq_[a-z_]+)\s*\(", hdr)) - inline)


def test_header_declares_exports_list():
    assert declared_symbols() == sorted(E.EXPORTS)


def test_library_exports_all_symbols():
    L = E.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert L.mq_abi_version() == 9


def test_errors_are_reported():
    eng = E.Engine()
    with pytest.raises(E.EngineError):
        eng.subscribe("a/b", 1, 1, qos=3)


SEGS = ["a", "b", "c", "", "+", "#", "$SYS", "$share", "$SHARE", "$ſhare", "g",
        "averyveryverylongsegment", "averyveryverylongsegmenz", "x"]


def rand_filter(r):
    return "/".join(r.choice(SEGS) for _ in range(r.randint(1, 5)))


@pytest.mark.parametrize("seed", range(6))
def test_update_semantics_match_oracle(seed):
    r = random.Random(seed)
    eng = E.Engine()
    orc = O.OracleIndex()
    cids, fids = {}, {}
    cid = lambda c: cids.setdefault(c, len(cids))
    fid = lambda f: fids.setdefault(f, len(fids))
    clients = [f"c{i}" for i in range(6)]
    filters = [rand_filter(r) for _ in range(40)]
    handle = 0
    for step in range(1500):
        op = r.random()
        f = r.choice(filters)
        c = r.choice(clients)
        if op < 0.40:
            qos, ident, flags = r.randint(0, 2), r.choice([0, 0, 5, 77]), r.randint(0, 15)
            a = eng.subscribe(f, cid(c), fid(f), qos, flags, ident)
            b = orc.subscribe(c, f, qos, ident, bool(flags & 1), bool(flags & 2), (flags >> 2) & 3,
                              client_id=cid(c), filter_id=fid(f))
            assert bool(a) == b, (step, "subscribe", f, c)
        elif op < 0.65:
            a = eng.unsubscribe(f, cid(c))
            b = orc.unsubscribe(f, c)
            assert bool(a) == b, (step, "unsubscribe", f, c)
        elif op < 0.75:
            i = r.randint(1, 4)
            assert bool(eng.inline_subscribe(f, i, fid(f))) == orc.inline_subscribe(f, i, fid(f))
        elif op < 0.82:
            i = r.randint(1, 4)
            assert bool(eng.inline_unsubscribe(f, i)) == orc.inline_unsubscribe(i, f)
        elif op < 0.95:
            t = f.replace("+", "p").replace("#", "h") if r.random() < 0.8 else f
            handle += 1
            plen, ret = r.choice([0, 5]), r.random() < 0.8
            assert eng.retain_message(t, handle, plen, ret) == orc.retain_message(t, handle, plen, ret)
        else:
            t = f.replace("+", "p").replace("#", "h")
            eng.retained_delete(t)
            orc.retained_delete(t)
        assert eng.retained_len() == orc.retained_len()
        if step % 50 == 0:
            assert eng.stats()["nodes"] == orc.particle_count(), step
            eng.check()
    st = eng.stats()
    assert st["nodes"] == orc.particle_count()
    assert (st["partners"] == 0) == (st["subs_merge"] == 0)


def test_partner_links_symmetric():
    """Every may-merge subscription has >= 1 partner and links are symmetric: a client with
    k pairwise co-matchable filters holds k*(k-1) links."""
    eng = E.Engine()
    for i, f in enumerate(["a/#", "a/b", "a/+", "x/y"]):
        eng.subscribe(f, 7, i, 0, 0, 0)
    st = eng.stats()
    assert st["subs_merge"] == 3 and st["partners"] == 6
    eng.check()
    eng.unsubscribe("a/#", 7)
    eng.check()
    st = eng.stats()
    assert st["subs_merge"] == 2 and st["partners"] == 2  # a/b ~ a/+ remain partners
    eng.unsubscribe("a/+", 7)
    st = eng.stats()
    assert st["subs_merge"] == 0 and st["partners"] == 0


def test_bulk_subscribe_matches_oracle():
    from mqmatch import workload as W
    w = W.gen_subscriptions(20000, 2000)
    eng = E.Engine()
    orc = O.OracleIndex()
    a = eng.subscribe_bulk(w)
    b = orc.subscribe_bulk(w)
    assert (a == b).all()
    st = eng.stats()
    assert st["nodes"] == orc.particle_count()
    assert st["subs"] + st["shared"] == int(a.sum())
    eng.check()


def test_partner_links_survive_churn():
    """Random unsubscribe / resubscribe churn on a workload index: after every round the
    device partner links name each partner's current slot (mq_index_check)."""
    from mqmatch import workload as W
    w = W.gen_subscriptions(20000, 600, seed=9)  # ~33 filters per client: many partners
    eng = E.Engine()
    eng.subscribe_bulk(w)
    eng.check()
    fs = W.strings(w["bytes"], w["offs"])
    r = random.Random(10)
    for _ in range(4):
        for _ in range(1500):
            i = r.randrange(len(fs))
            if r.random() < 0.5:
                eng.unsubscribe(fs[i], int(w["client_ids"][i]))
            else:
                eng.subscribe(fs[i], r.randrange(600), int(w["filter_ids"][i]), 1, 0, 3)
        eng.check()
    assert eng.stats()["subs_merge"] > 0


def test_unsubscribe_everything_empties_trie():
    from mqmatch import workload as W
    w = W.gen_subscriptions(3000, 300, seed=7)
    eng = E.Engine()
    eng.subscribe_bulk(w)
    fs = W.strings(w["bytes"], w["offs"])
    for i, f in enumerate(fs):
        eng.unsubscribe(f, int(w["client_ids"][i]))
    st = eng.stats()
    assert st["nodes"] == 0 and st["subs"] == 0 and st["shared"] == 0 and st["subs_merge"] == 0
    assert st["partners"] == 0


def test_options_without_device():
    """mq_set_option is accepted before the device exists (applied when it is first touched) and
    rejects unknown options."""
    eng = E.Engine()
    eng.set_option(E.OPT_CHUNK_ROWS, 1 << 20)
    eng.set_option(E.OPT_PATCH_CAP, 1024)
    eng.set_option(E.OPT_MAX, 0)  # (the newest option: the range check admits it)
    with pytest.raises(E.EngineError):
        eng.set_option(99, 1)
    with pytest.raises(E.EngineError):
        eng.set_option(E.OPT_MAX + 1, 1)


def test_edge_load_option():
    """MQ_OPT_EDGE_LOAD 16 (the default) keeps the edge table at most a sixteenth full, 2 at most half;
    other values are rejected; answers are unchanged."""
    from mqmatch import workload as W
    w = W.gen_subscriptions(20000, 2000, seed=71)
    sparse, dense = E.Engine(), E.Engine()
    dense.set_option(E.OPT_EDGE_LOAD, 2)
    with pytest.raises(E.EngineError):
        sparse.set_option(E.OPT_EDGE_LOAD, 3)
    assert (sparse.subscribe_bulk(w) == dense.subscribe_bulk(w)).all()
    s, d = sparse.stats(), dense.stats()
    assert s["edges"] == d["edges"] and s["edges"] * 16 <= s["edge_capacity"]
    assert s["edge_capacity"] > d["edge_capacity"]
    sparse.check()
    for c in range(300):  # per-entry growth keeps the bound
        assert sparse.subscribe(f"x/{c}/y/{c % 7}", c, 0, 1, 0, 0) == dense.subscribe(f"x/{c}/y/{c % 7}", c, 0, 1, 0, 0)
    s = sparse.stats()
    assert s["edges"] * 16 <= s["edge_capacity"]
    sparse.check()


@pytest.mark.parametrize("n_shards", [1, 2])
def test_merge_records_update_in_place(n_shards):
    """Nodes with at least Index::kIncLinks (256) partner links update their merge records in
    place (flush_merge -> merge_patch): the changed slots come off the pair lists and go back
    on. Hot nodes here: '#', 'a/+', 'a/b' and 'a/#' shared by 400 clients. Every round mixes new
    and dropped partners, Qos / NoLocal / identifier changes (the partners' links and the pair
    slots copy them), direct subscriptions coming and going (merge slots move within the list)
    and lists outgrowing their slabs; after each, mq_index_check holds — every link and pair
    entry current and nothing stale left on a list — on every shard."""
    r = random.Random(40 + n_shards)
    filters = ["#", "a/+", "a/b", "a/#", "x/y", "x/+", "q/r/s", "+/b"]
    engs = [E.Engine(shard=k, n_shards=n_shards) for k in range(n_shards)]
    state = {}
    for c in range(400):
        for f in r.sample(filters, 3):
            state[(c, f)] = True
            for e in engs:
                e.subscribe(f, c, filters.index(f), r.randint(0, 2), 0, 0)
    for e in engs:
        e.check()
    for rnd in range(6):
        for _ in range(800):
            c, f = r.randrange(460), r.choice(filters)
            if r.random() < 0.4 and (c, f) in state:
                del state[(c, f)]
                for e in engs:
                    e.unsubscribe(f, c)
            else:
                state[(c, f)] = True
                q, fl, ident = r.randint(0, 2), r.choice([0, 1]), r.choice([0, 0, 5])
                for e in engs:
                    e.subscribe(f, c, filters.index(f), q, fl, ident)
        for e in engs:
            e.check()
    assert sum(e.stats()["subs_merge"] for e in engs) > 500


def test_header_compiles_as_c(tmp_path):
    """include/mqmatch.h (with its inline mq_topic_patch) is plain C99: what cgo compiles."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "h.c"
    src.write_text('#include "mqmatch.h"\nint main(void) { return (int)MQ_ABI_VERSION - 9; }\n')
    r = subprocess.run([cc, "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(REPO, "include"), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_host_topic_patches_resolves_own_and_set_patches():
    """host_topic_patches (the Python form of mq_topic_patch) on a hand-built host result: a topic
    with its own patches, and two topics of one merge set whose set patches (x << 26 | k) land on
    their own rows through their packed merge rows."""
    import numpy as np
    dt = E._TOPIC_SPANS_DT
    t = np.zeros(3, dt)
    t["n_rows"] = [10, 20, 30]
    t["patch_base"], t["n_patches"], t["flags"] = [0, 0, 0], [2, 2, 2], [0, 1, 1]
    a = {"topics": t,
         "patches": np.array([[3, 7], [5, 9]], np.uint32),
         "set_patches": np.array([[0 << 26 | 1, 11], [1 << 26 | 2, 12]], np.uint32),
         "merge_rows": np.array([4, 8, 0, 0, 20, 25], np.uint32),   # topic 1: rows 4, 8; topic 2: 20, 25
         "merge_base": np.array([0, 0, 4], np.uint32)}
    tid, row, meta = E.host_topic_patches(a)
    got = sorted(zip(tid.tolist(), row.tolist(), meta.tolist()))
    assert got == [(0, 3, 7), (0, 5, 9), (1, 5, 11), (1, 10, 12), (2, 21, 11), (2, 27, 12)]
