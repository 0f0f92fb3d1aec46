"""Generate tests/golden/topics_golden.json: a fixed scenario of TopicsIndex updates and queries
with the expected results of the CPU restatement (oracle/, pinned by the reference's own
known-answer tests in tests/kat_cases.py). The reference is Go and cannot run here (SURVEY.md
§8c); these vectors freeze the restatement's answers so that the oracle cannot drift and the
HIP engine is checked against data, not only against live oracle calls.

  python tests/golden/make_golden.py      # rewrites topics_golden.json

Scenario (seeded): subscriptions with '+'/'#' at every level, empty segments, long (hashed)
segments, $SYS / $foo topics (Q3/Q4), $share groups with mixed-case prefixes (Q9), repeated
subscribes (overwrite), unsubscribes (Q10), inline subscriptions (Q2/Q8), retained messages with
deletes and empty payloads (Q5/Q6/Q12/Q15), and Messages filters.
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))

SEGS = ["a", "b", "c", "", "x", "$SYS", "$foo", "averyveryverylongsegment-xyz", "ü", "d"]


def rand_topic(r, wild):
    n = r.randint(1, 5)
    out = []
    for i in range(n):
        t = r.random()
        if wild and t < 0.2:
            out.append("+")
        elif wild and t < 0.3 and i == n - 1:
            out.append("#")
        else:
            s = r.choice(SEGS)
            if i > 0 and s.startswith("$"):
                s = "y"
            out.append(s)
    return "/".join(out)


def scenario(seed=0x601DE):
    r = random.Random(seed)
    ops = []
    clients = [f"cl{i}" for i in range(40)]
    for _ in range(400):
        f = rand_topic(r, True)
        if r.random() < 0.1:
            f = r.choice(["$share", "$SHARE", "$Share"]) + f"/g{r.randrange(3)}/" + rand_topic(r, True)
        ops.append(["sub", r.choice(clients), f, r.randrange(3), r.choice([0, 0, r.randrange(1, 100)]),
                    r.random() < 0.1, r.random() < 0.5, r.randrange(3)])
    for _ in range(40):
        ops.append(["unsub", r.choice(clients), rand_topic(r, True)])
    for i in range(30):
        ops.append(["inline", rand_topic(r, True), r.randrange(1, 12)])
    for i in range(120):
        ops.append(["retain", rand_topic(r, False), 1000 + i, r.choice([5, 5, 5, 0]), r.random() < 0.9])
    for _ in range(10):
        ops.append(["retdel", rand_topic(r, False)])
    topics = sorted({rand_topic(r, False) for _ in range(300)} | {"$SYS/x", "$foo/a", "a", "a/b", "/a", "a//b", "a/"})
    filters = sorted({rand_topic(r, True) for _ in range(120)} | {"#", "+", "+/#", "a/#", "$SYS/#", "x/#"})
    return ops, topics, filters


def replay(ix, ops):
    rets = []
    for op in ops:
        if op[0] == "sub":
            _, c, f, q, i, nl, rap, rh = op
            rets.append(ix.subscribe(c, f, qos=q, identifier=i, no_local=nl, rap=rap, rh=rh))
        elif op[0] == "unsub":
            rets.append(ix.unsubscribe(op[2], op[1]))
        elif op[0] == "inline":
            rets.append(ix.inline_subscribe(op[1], op[2]))
        elif op[0] == "retain":
            _, t, h, plen, retain = op
            rets.append(ix.retain_message(t, payload=b"p" * plen, retain=retain, handle=h)[0])
        elif op[0] == "retdel":
            ix.retained_delete(op[1])
            rets.append(None)
    return [r if r is None or isinstance(r, bool) else int(r) for r in rets]


def jsonable(s):
    return {"subscriptions": s["subscriptions"], "shared": s["shared"],
            "inline": {str(k): v for k, v in s["inline"].items()}}


def main():
    from adapters import OracleAdapter
    ops, topics, filters = scenario()
    ix = OracleAdapter()
    rets = replay(ix, ops)
    out = {"generator": "tests/golden/make_golden.py (oracle/ C++ restatement of topics.go)",
           "ops": ops, "returns": rets, "topics": topics, "filters": filters,
           "subscribers": [jsonable(ix.subscribers(t)) for t in topics],
           "messages": [sorted(int(h) for h in ix.messages(f)) for f in filters]}
    with open(os.path.join(HERE, "topics_golden.json"), "w") as fh:
        json.dump(out, fh, indent=0, sort_keys=True, ensure_ascii=False)
    print(f"{len(ops)} ops, {len(topics)} topics, {len(filters)} filters")


if __name__ == "__main__":
    main()
