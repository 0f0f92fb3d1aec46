"""The oracle (CPU restatement of the Go TopicsIndex) against the reference's own known-answer
tests — this pins the oracle (the Go toolchain is absent, so the reference
cannot be run here). CPU only."""
import pytest

import oracle as O
from adapters import OracleAdapter
from kat_cases import KATS, MESSAGE_KATS


@pytest.mark.parametrize("kat", KATS + MESSAGE_KATS, ids=lambda f: f.__name__)
def test_oracle_kat(kat):
    kat(OracleAdapter)


def test_isolate_particle():  # topics_test.go:452-482
    cases = [("path/to/my/mqtt", 0, "path", True), ("path/to/my/mqtt", 1, "to", True),
             ("path/to/my/mqtt", 2, "my", True), ("path/to/my/mqtt", 3, "mqtt", False),
             ("/path/", 0, "", True), ("/path/", 1, "path", True), ("/path/", 2, "", False),
             ("a/b/c/+/+", 3, "+", True), ("a/b/c/+/+", 4, "+", False)]
    for f, d, want, hn in cases:
        assert O.isolate_particle(f, d) == (want, hn), (f, d)
    # beyond the last level: the last segment again (relied on by set(filter, 2), Q13)
    assert O.isolate_particle("a/b", 5) == ("b", False)
    assert O.isolate_particle("a", 2) == ("a", False)


def test_is_valid_filter():  # topics_test.go:755-771
    assert O.is_valid_filter("a/b/c", False)
    assert O.is_valid_filter("a/b//c", False)
    assert O.is_valid_filter("$SYS", False)
    assert O.is_valid_filter("$SYS/info", False)
    assert O.is_valid_filter("$sys/info", False)
    assert O.is_valid_filter("abc/#", False)
    assert not O.is_valid_filter("", False)
    for f in ["$SHARE", "$SHARE/", "$SHARE/b+/", "$SHARE/+", "$SHARE/#", "$SHARE/#/", "a/#/c"]:
        assert not O.is_valid_filter(f, False), f


def test_is_valid_for_publish():  # topics_test.go:773-779
    assert O.is_valid_filter("", True)
    assert O.is_valid_filter("a/b/c", True)
    assert not O.is_valid_filter("a/b/+/d", True)
    assert not O.is_valid_filter("a/b/#", True)
    assert not O.is_valid_filter("$SYS/info", True)


def test_is_shared_filter():  # topics_test.go:781-784
    assert O.is_shared_filter("$SHARE/tmp/a/b/c")
    assert not O.is_shared_filter("a/b/c")


def test_equal_fold_unicode():
    """strings.EqualFold's Unicode simple folding (Q9). No reference test pins this; the
    expectations follow Go's documented folding (ſ U+017F folds with s/S; K U+212A with k)."""
    assert O.equal_fold("$share", "$SHARE")
    assert O.equal_fold("$ShArE", "$SHARE")
    assert O.equal_fold("$ſhare", "$SHARE")
    assert not O.equal_fold("$shar", "$SHARE")
    assert not O.equal_fold("$sharé", "$SHARE")
    assert O.equal_fold("K", "k")
    assert O.is_shared_filter("$ſHARE/g/a")


def test_share_with_unicode_prefix_routes_shared():
    ix = OracleAdapter()
    ix.subscribe("c1", "$ſhare/g/a/b")
    s = ix.subscribers("a/b")
    assert s["subscriptions"] == {} and list(s["shared"]) == ["$ſhare/g/a/b"]


def test_index_set_seek_trim_restated():  # topics_test.go:339-399 through the public API
    ix = OracleAdapter()
    ix.subscribe("cl1", "a/b/c")
    ix.subscribe("cl1", "a/b/c/d/e/f")
    ix.subscribe("cl1", "a/b")
    assert ix.path_exists("a/b/c/d/e/f") and not ix.path_exists("d/e/f")
    ix.unsubscribe("a/b/c/d/e/f", "cl1")
    assert not ix.path_exists("a/b/c/d") and ix.path_exists("a/b/c")
    ix.unsubscribe("a/b/c", "cl1")
    ix.unsubscribe("a/b", "cl1")
    assert not ix.path_exists("a")
    ix.subscribe("x", "/c")  # TestIndexSetPrefixed
    assert ix.path_exists("/c")


def test_merge_shared_selected_host():  # topics_test.go:568-588 (host-side, Python mirror)
    from mqmatch.engine import Subscribers, Subscription
    s = Subscribers(
        shared_selected={"cl1": Subscription("$SHARE/tmp/a/b/c", 110, 1),
                         "cl2": Subscription("$SHARE/tmp2/a/b/c", 111, 1)},
        subscriptions={"cl2": Subscription("a/b/c", 112, 1)})
    s.merge_shared_selected()
    assert set(s.subscriptions) == {"cl1", "cl2"}
    assert s.subscriptions["cl2"].identifiers == {"$SHARE/tmp2/a/b/c": 111, "a/b/c": 112}


def test_select_shared_host():  # topics_test.go:552-566 (the pick)
    from mqmatch.engine import Subscribers, Subscription
    s = Subscribers(shared={"$SHARE/tmp/a/b/c": {"cl1": Subscription("$SHARE/tmp/a/b/c", 110, 1),
                                                  "cl1b": Subscription("$SHARE/tmp/a/b/c", 111),
                                                  "cl2": Subscription("$SHARE/tmp/a/b/c", 112)},
                            "$SHARE/tmp2/a/b/c": {"cl3": Subscription("$SHARE/tmp2/a/b/c", 113)}})
    s.select_shared()
    assert len(s.shared_selected) == 2


def test_retained_expiry_keeps_path():
    """Q12: Retained.Delete (server.go:1726) drops the map entry; the particle keeps its
    retainPath, so Messages no longer returns it but the path survives trims."""
    ix = OracleAdapter()
    ix.retain_message("a/b", b"x")
    ix.subscribe("c", "a/b")
    ix.retained_delete("a/b")
    assert ix.messages("a/+") == [] and ix.messages("a/b") == []
    ix.unsubscribe("a/b", "c")
    assert ix.path_exists("a/b")  # retainPath still set


def test_match_topic():  # hooks/auth/ledger_test.go:461-493 (auth.MatchTopic)
    cases = [("a/+/c/+", "a/b/c/d", ["b", "d"], True), ("a/+/+/+", "a/b/c/d", ["b", "c", "d"], True),
             ("stuff/#", "stuff/things/yeah", ["things/yeah"], True),
             ("a/+/#/+", "a/b/c/d/as/dds", ["b", "c/d/as/dds"], True), ("test", "test", [], True),
             ("things/stuff//", "things/stuff/", [], False), ("t", "t2", [], False), (" ", "  ", [], False)]
    for f, t, el, m in cases:
        assert O.match_topic(f, t) == (el, m), (f, t)


def test_fast_baseline_matches_oracle():
    """The CPU baseline's fast restatement (oracle/topics_fast.h) gives the oracle's digests on a
    workload batch, including '$' topics, shared and inline subscriptions."""
    import random
    import numpy as np
    from mqmatch import workload as W
    w = W.gen_subscriptions(30000, 3000, seed=91)
    orc = O.OracleIndex()
    orc.subscribe_bulk(w)
    r = random.Random(92)
    for i in range(200):  # inline subscriptions with repeated ids (last write wins)
        f = "/".join(r.choice(["a", "+", "#", "b"]) for _ in range(r.randint(1, 3)))
        orc.inline_subscribe(f, r.randint(1, 20))
    tb, to = W.gen_topics(w, 4000, seed=93)
    extra = ["a", "a/b", "b/a/x", "$SYS/a", "", "a/+"]
    topics = W.strings(tb, to) + extra
    raw = [t.encode("utf-8", "surrogateescape") for t in topics]
    offs = np.zeros(len(raw) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in raw])
    b = np.frombuffer(b"".join(raw) + b"\0" * 16, np.uint8).copy()
    od, ocnt, _ = orc.digest_batch(b, offs, nthreads=4)
    fd, fcnt = orc.fast().digest_batch(b, offs, nthreads=4)
    assert (fcnt == ocnt).all()
    assert (fd == od).all(), np.nonzero(fd != od)[0][:5]
    assert ocnt[:, 0].sum() > len(topics) and ocnt[:, 3].sum() > 0


def test_fast_messages_baseline_matches_oracle():
    """The Messages CPU baseline's fast restatement (oracle/topics_fast.h, FastMsgIndex) gives the
    oracle's digests: a config-5-shaped workload plus the Q4 ($SYS at level 0), Q5 (x/# excludes x)
    and Q6 (a retained "" entry, particles without a retain path) corners."""
    import random
    import numpy as np
    from mqmatch import workload as W
    rb, ro, hd, rh = W.gen_retained(20000, n_sys=200, seed=94)
    fb, fo = W.gen_msg_filters(rh, 2000, seed=95)
    orc = O.OracleIndex()
    orc.retain_bulk(rb, ro, hd)
    r = random.Random(96)
    h = 10 ** 9
    for t in ["", "q/r", "q/r/s", "$SYS/x/y", "a/$SYS"]:
        h += 1
        orc.retain_message(t, h, 1, True)
    for f in ["q/z", "zz/top"]:  # subscription-only particles (no retain path)
        orc.subscribe("c1", f)
    extra = ["#", "+", "+/+", "$SYS/#", "+/$SYS/#", "q/#", "q/+", "q/r", "q/z", "zz/+", "+/z", "", "q/+/#",
             "/".join(r.choice(["+", "#", "q", "r"]) for _ in range(3))]
    filters = W.strings(fb, fo) + extra
    raw = [f.encode("utf-8", "surrogateescape") for f in filters]
    offs = np.zeros(len(raw) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in raw])
    b = np.frombuffer(b"".join(raw) + b"\0" * 16, np.uint8).copy()
    od, ocnt, _ = orc.messages_digest_batch(b, offs, nthreads=4)
    fd, fcnt = orc.fast_messages().digest_batch(b, offs, nthreads=4)
    assert (fcnt == ocnt).all(), np.nonzero(fcnt != ocnt)[0][:5]
    assert (fd == od).all(), np.nonzero(fd != od)[0][:5]
    assert ocnt.sum() > len(filters)
