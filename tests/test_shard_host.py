"""The sharded index's host side (CPU; mq_config.shard_count > 1): every update
goes to every shard; the shards' answers combine to the reference's (the owner answers
Subscribe / InlineSubscribe / RetainMessage, the others return 0; Unsubscribe /
InlineUnsubscribe are the OR of "particle exists" over shards, Q10), and each shard's image
keeps its invariants, cross-shard merge partners included (mq_index_check)."""
import random

import pytest

from mqmatch import engine as E
import oracle as O

SEGS = ["a", "b", "c", "", "+", "#", "$SYS", "$share", "$SHARE", "g", "x", "longersegment-abcdefghijk"]


def _filter(r):
    return "/".join(r.choice(SEGS) for _ in range(r.randint(1, 5)))


@pytest.mark.parametrize("n_shards", [2, 3, 5])
def test_sharded_updates_match_oracle(n_shards):
    r = random.Random(300 + n_shards)
    shards = [E.Engine(shard=k, n_shards=n_shards) for k in range(n_shards)]
    orc = O.OracleIndex()
    fids, cids = {}, {}
    fid = lambda f: fids.setdefault(f, len(fids))
    cid = lambda c: cids.setdefault(c, len(cids))
    live = []
    for step in range(3000):
        op = r.random()
        if op < 0.55 or not live:
            f, c = _filter(r), f"c{r.randrange(40)}"
            q, ident, nl = r.randint(0, 2), r.choice([0, 0, 3, 7]), r.random() < 0.2
            got = [e.subscribe(f, cid(c), fid(f), q, 1 if nl else 0, ident) for e in shards]
            assert sum(1 for g in got if g == 1) <= 1
            assert any(got) == orc.subscribe(c, f, q, ident, nl, client_id=cid(c), filter_id=fid(f)), (step, f)
            live.append((f, c))
        elif op < 0.80:
            f, c = r.choice(live) if r.random() < 0.8 else (_filter(r), f"c{r.randrange(40)}")
            got = [e.unsubscribe(f, cid(c)) for e in shards]
            assert any(got) == orc.unsubscribe(f, c), (step, f)
        elif op < 0.88:
            f, i = _filter(r), r.randint(1, 9)
            got = [e.inline_subscribe(f, i, fid(f)) for e in shards]
            assert any(got) == orc.inline_subscribe(f, i, filter_id=fid(f)), (step, f)
        elif op < 0.93:
            f, i = _filter(r), r.randint(1, 9)
            got = [e.inline_unsubscribe(f, i) for e in shards]
            assert any(got) == orc.inline_unsubscribe(i, f), (step, f)
        else:
            t = "/".join(r.choice(["a", "b", "x", "", "$SYS"]) for _ in range(r.randint(1, 4)))
            pl = 0 if r.random() < 0.3 else 5
            got = [e.retain_message(t, step + 1, pl, True) for e in shards]
            assert sum(got) == orc.retain_message(t, step + 1, pl, True), (step, t)
        if step % 500 == 499:
            for e in shards:
                e.check()  # partner links (foreign ones included), pair blocks, lists
    for e in shards:
        e.check()
    st = [e.stats() for e in shards]
    assert sum(s["foreign"] for s in st) > 0 and sum(s["subs"] for s in st) > 0
    assert sum(e.retained_len() for e in shards) == orc.retained_len()


def test_shard_config_validation():
    with pytest.raises(E.EngineError):
        E.Engine(shard=3, n_shards=2)
    with pytest.raises(E.EngineError):
        E.Engine(shard=0, n_shards=17)


def test_sharded_bulk_build_parallel():
    """The parallel bulk build of a sharded index (its DFS rank keys are set on many threads) on
    a fresh and on an emptied index: every shard keeps its invariants, and together they hold
    every subscription once (a dirty-page list once grew from several threads: heap corruption)."""
    from mqmatch import workload as W
    w = W.gen_subscriptions(200000, 20000, seed=91)
    shards = [E.Engine(shard=k, n_shards=4) for k in range(4)]
    owned = sum(int(e.subscribe_bulk(w).sum()) for e in shards)
    for e in shards:
        e.check()
    assert owned == sum(e.stats()["subs"] + e.stats()["shared"] for e in shards)
