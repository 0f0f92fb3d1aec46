"""Known-answer tests transcribed from the reference's own test suite for the TopicsIndex path
(/root/reference/topics_test.go, server_test.go). Each function takes an index adapter
(tests/adapters.py) and asserts the reference's expectations; white-box assertions on
`index.root.particles` are restated through the public API.
"""
SHARE = "$SHARE"


def kat_subscribe(mk):  # topics_test.go:170-226
    ix = mk()
    assert ix.subscribe("cl1", "a/b/c", qos=2) is True
    assert ix.subscribe("cl1", "a/b/c", qos=1) is False
    assert ix.subscribe("cl1", "A/B/c", qos=1) is True
    assert ix.subscribe("cl1", "d/+") is True
    assert ix.subscribe("cl1", "d/e/#") is True
    s = ix.subscribers("a/b/c")
    assert s["subscriptions"]["cl1"]["qos"] == 1  # the replaced subscription's Qos


def kat_subscribe_shared(mk):  # topics_test.go:228-238
    ix = mk()
    ix.subscribe("cl1", SHARE + "/tmp/a/b/c", qos=2)
    s = ix.subscribers("a/b/c")
    assert s["subscriptions"] == {}
    assert list(s["shared"]) == [SHARE + "/tmp/a/b/c"]
    assert s["shared"][SHARE + "/tmp/a/b/c"]["cl1"]["qos"] == 2


def kat_unsubscribe(mk):  # topics_test.go:254-297
    ix = mk()
    ix.subscribe("cl1", "a/b/c/d", qos=1)
    ix.subscribe("cl1", "a/b/+/d", qos=1)
    ix.subscribe("cl1", "d/e/f", qos=1)
    ix.subscribe("cl2", "d/e/f", qos=1)
    ix.subscribe("cl3", "#", qos=2)
    assert ix.unsubscribe("a/b/c/d", "cl1") is True
    s = ix.subscribers("a/b/c/d")
    assert set(s["subscriptions"]) == {"cl1", "cl3"}
    assert s["subscriptions"]["cl1"]["filter"] == "a/b/+/d"
    assert ix.unsubscribe("d/e/f", "cl1") is True
    s = ix.subscribers("d/e/f")
    assert set(s["subscriptions"]) == {"cl2", "cl3"}
    assert ix.unsubscribe("fdasfdas/dfsfads/sa", "nobody") is False


def kat_unsubscribe_no_cascade(mk):  # topics_test.go:299-311
    ix = mk()
    ix.subscribe("cl1", "a/b/c")
    ix.subscribe("cl1", "a/b/c/e/e")
    assert ix.unsubscribe("a/b/c/e/e", "cl1") is True
    assert set(ix.subscribers("a/b/c")["subscriptions"]) == {"cl1"}
    assert ix.subscribers("a/b/c/e/e")["subscriptions"] == {}


def kat_unsubscribe_shared(mk):  # topics_test.go:313-326
    ix = mk()
    ix.subscribe("cl1", "$SHARE/tmp/a/b/c", qos=2)
    assert ix.subscribers("a/b/c")["shared"]["$SHARE/tmp/a/b/c"]["cl1"]["qos"] == 2
    assert ix.unsubscribe("$share/tmp/a/b/c", "cl1") is True
    assert ix.subscribers("a/b/c")["shared"] == {}


def kat_retain_message(mk):  # topics_test.go:408-443
    ix = mk()
    r, _ = ix.retain_message("a/b/c", b"hello", True)
    assert r == 1
    assert ix.retained_len() == 1
    r, _ = ix.retain_message("a/b/d/f", b"hello", True)
    assert r == 1
    r, _ = ix.retain_message("a/b/d/f", b"hello", True)
    assert r == 1
    r, _ = ix.retain_message("a/b/c", b"", False)
    assert r == -1
    assert ix.retained_len() == 1
    r, _ = ix.retain_message("a/b/c", b"", False)
    assert r == 0


def kat_scan_subscribers(mk):  # topics_test.go:490-528
    ix = mk()
    ix.subscribe("cl1", "a/b/c", qos=1, identifier=22)
    ix.subscribe("cl1", "a/b/c/d/e/f", qos=1)
    ix.subscribe("cl1", "a/b/c/d/+/f", qos=2)
    ix.subscribe("cl2", "a/#", qos=0)
    ix.subscribe("cl2", "a/b/c", qos=1)
    ix.subscribe("cl2", "a/b/+", qos=2, identifier=77)
    ix.subscribe("cl2", "d/e/f", qos=2, identifier=7237)
    ix.subscribe("cl2", "$SYS/uptime", qos=2, identifier=3)
    ix.subscribe("cl3", "+/b", qos=1, identifier=234)
    ix.subscribe("cl4", "#", qos=0, identifier=5)
    ix.subscribe("cl2", "$SYS/test", qos=0, identifier=2)
    s = ix.subscribers("a/b/c")["subscriptions"]
    assert set(s) == {"cl1", "cl2", "cl4"}
    assert s["cl1"]["qos"] == 1 and s["cl2"]["qos"] == 2 and s["cl4"]["qos"] == 0
    # Go map lookups return the zero value for a missing key (require.Equal(t, 0, m[k]))
    assert s["cl1"]["identifiers"].get("a/b/c", 0) == 22
    assert s["cl2"]["identifiers"].get("a/#", 0) == 0
    assert s["cl2"]["identifiers"].get("a/b/+", 0) == 77
    assert s["cl2"]["identifiers"].get("a/b/c", 0) == 0
    assert s["cl4"]["identifiers"].get("#", 0) == 5
    s = ix.subscribers("d/e/f/g")["subscriptions"]
    assert set(s) == {"cl4"} and s["cl4"]["qos"] == 0 and s["cl4"]["identifiers"].get("#", 0) == 5
    assert ix.subscribers("")["subscriptions"] == {}


def kat_inheritance_bug(mk):  # topics_test.go:530-537
    ix = mk()
    ix.subscribe("cl1", "a/b/c")
    ix.subscribe("cl2", "a/b")
    assert len(ix.subscribers("a/b/c")["subscriptions"]) == 1


def kat_scan_shared(mk):  # topics_test.go:539-550
    ix = mk()
    ix.subscribe("cl1", SHARE + "/tmp/a/b/c", qos=1, identifier=111)
    ix.subscribe("cl2", SHARE + "/tmp/a/b/c", qos=0, identifier=112)
    ix.subscribe("cl3", SHARE + "/tmp2/a/b/c", qos=0, identifier=113)
    ix.subscribe("cl2", SHARE + "/tmp/a/b/+", qos=0, identifier=10)
    ix.subscribe("cl3", SHARE + "/tmp/a/b/+", qos=1, identifier=200)
    ix.subscribe("cl4", SHARE + "/tmp/a/b/+", qos=0, identifier=201)
    ix.subscribe("cl5", SHARE + "/tmp/a/b/c/#", qos=0)
    assert len(ix.subscribers("a/b/c")["shared"]) == 4


def kat_select_shared(mk):  # topics_test.go:552-566 (the Shared side; the pick is host-side)
    ix = mk()
    ix.subscribe("cl1", SHARE + "/tmp/a/b/c", qos=1, identifier=110)
    ix.subscribe("cl1b", SHARE + "/tmp/a/b/c", qos=0, identifier=111)
    ix.subscribe("cl2", SHARE + "/tmp/a/b/c", qos=0, identifier=112)
    ix.subscribe("cl3", SHARE + "/tmp2/a/b/c", qos=0, identifier=113)
    sh = ix.subscribers("a/b/c")["shared"]
    assert set(sh) == {SHARE + "/tmp/a/b/c", SHARE + "/tmp2/a/b/c"}
    assert len(sh[SHARE + "/tmp/a/b/c"]) == 3 and len(sh[SHARE + "/tmp2/a/b/c"]) == 1


# topics_test.go:590-625 — filter, topic, matched
SUBSCRIBERS_FIND = [
    ("a", "a", True), ("a/", "a", False), ("a/", "a/", True), ("/a", "/a", True),
    ("path/to/my/mqtt", "path/to/my/mqtt", True), ("path/to/+/mqtt", "path/to/my/mqtt", True),
    ("+/to/+/mqtt", "path/to/my/mqtt", True), ("#", "path/to/my/mqtt", True),
    ("+/+/+/+", "path/to/my/mqtt", True), ("+/+/+/#", "path/to/my/mqtt", True),
    ("zen/#", "zen", True), ("trailing-end/#", "trailing-end/", True),
    ("+/prefixed", "/prefixed", True), ("+/+/#", "path/to/my/mqtt", True),
    ("path/to/", "path/to/my/mqtt", False), ("#/stuff", "path/to/my/mqtt", False),
    ("#", "$SYS/info", False), ("$SYS/#", "$SYS/info", True), ("+/info", "$SYS/info", False),
]


def kat_subscribers_find(mk):
    for f, t, matched in SUBSCRIBERS_FIND:
        ix = mk()
        ix.subscribe("cl1", f)
        assert (len(ix.subscribers(t)["subscriptions"]) == 1) == matched, (f, t)


# topics_test.go:640-685 — retained topics x filters -> counts
MESSAGES_TOPICS = ["$SYS/uptime", "$SYS/info", "a/b/c/d", "a/b/c/e", "a/b/d/f", "q/w/e/r/t/y",
                   "q/x/e/r/t/o", "asdf"]
MESSAGES_PATTERN = [("a/b/c/d", 1), ("$SYS/+", 2), ("$SYS/#", 2), ("#", 6), ("a/b/c/+", 2),
                    ("a/+/c/+", 2), ("+/+/+/d", 1), ("q/w/e/#", 1), ("+/+/+/+", 3), ("q/#", 2),
                    ("asdf", 1), ("", 0), ("#", 6)]


def kat_messages_pattern(mk):
    ix = mk()
    for t in MESSAGES_TOPICS:
        ix.retain_message(t, b"hello", True)
    for f, n in MESSAGES_PATTERN:
        assert len(ix.messages(f)) == n, f


def kat_inline_subscribe(mk):  # topics_test.go:946-1001
    ix = mk()
    assert ix.inline_subscribe("a/b/c", 1) is True
    assert ix.inline_subscribe("a/b/c", 1) is False
    assert ix.inline_subscribe("a/b/c", 2) is True
    assert ix.inline_subscribe("A/B/c", 1) is True
    assert ix.inline_subscribe("d/+", 1) is True
    assert ix.inline_subscribe("d/e/#", 1) is True
    assert set(ix.subscribers("a/b/c")["inline"]) == {1, 2}


def kat_inline_unsubscribe(mk):  # topics_test.go:1003-1067
    ix = mk()
    ix.inline_subscribe("a/b/c/d", 1)
    ix.inline_subscribe("d/e/f", 1)
    ix.inline_subscribe("d/e/f", 2)
    ix.inline_subscribe("a/b/+/d", 1)
    ix.inline_subscribe("d/e/f", 1)
    ix.inline_subscribe("d/e/f", 1)
    ix.inline_subscribe("#", 1)
    assert ix.inline_unsubscribe(1, "a/b/c/d") is True
    inl = ix.subscribers("a/b/c/d")["inline"]
    assert set(inl) == {1}  # a/b/+/d (id 1) then # (id 1): last write is '#'
    assert inl[1]["filter"] == "#"
    assert ix.inline_unsubscribe(1, "d/e/f") is True
    assert set(ix.subscribers("d/e/f")["inline"]) == {1, 2}  # id 2 at d/e/f, id 1 from '#'
    assert ix.inline_unsubscribe(1, "not/exist") is False


def wire_subscription_ids(sub):
    """server.go:1036-1042: sorted Identifiers values; zero ids are not encoded
    (packets/properties.go, SubscriptionIdentifier)."""
    return [i for i in sorted(sub["identifiers"].values()) if i > 0]


def kat_publish_identifiers(mk):  # server_test.go:1973-1999 + packets/tpackets.go:1848-1872
    ix = mk()
    assert ix.subscribe("cl", "a/b/+", identifier=2) is True
    assert ix.subscribe("cl", "a/#", identifier=3) is True
    assert ix.subscribe("cl", "d/e/f", identifier=4) is True
    s = ix.subscribers("a/b/c")["subscriptions"]
    assert wire_subscription_ids(s["cl"]) == [2, 3]  # TPublishSubscriberIdentifier: 11,2, 11,3


def kat_publish_shared_group(mk):  # server_test.go:1882-1941 (candidates before the pick)
    ix = mk()
    assert ix.subscribe("cl1", "a/b/c") is True
    assert ix.subscribe("cl2", SHARE + "/tmp/a/b/c") is True
    assert ix.subscribe("cl3", SHARE + "/tmp/a/b/c") is True
    s = ix.subscribers("a/b/c")
    assert set(s["subscriptions"]) == {"cl1"}
    assert set(s["shared"][SHARE + "/tmp/a/b/c"]) == {"cl2", "cl3"}


def kat_publish_nolocal(mk):  # server_test.go:1857-1880 (NoLocal reaches publishToClient)
    ix = mk()
    assert ix.subscribe("cl1", "a/b/c", no_local=True) is True
    assert ix.subscribers("a/b/c")["subscriptions"]["cl1"]["no_local"] is True


KATS = [kat_subscribe, kat_subscribe_shared, kat_unsubscribe, kat_unsubscribe_no_cascade,
        kat_unsubscribe_shared, kat_retain_message, kat_scan_subscribers, kat_inheritance_bug,
        kat_scan_shared, kat_select_shared, kat_subscribers_find, kat_inline_subscribe,
        kat_inline_unsubscribe, kat_publish_identifiers, kat_publish_shared_group,
        kat_publish_nolocal]
MESSAGE_KATS = [kat_messages_pattern]
