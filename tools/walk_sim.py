"""Host-side model of the match walk's memory rounds and loads, for choosing the walk's design
(DESIGN.md §4.0): the level-synchronous frontier (k_walkf: one dependent round per topic level,
a literal probe per frontier particle and a walk-record load per '+' child) against a
prefix-hash walk (edges placed by the hash of the particle's whole path, so a branch's literal
continuation is probed at every remaining level at once: one round per nested '+' branch, but
speculative probes past the point where the chain breaks). Counts rounds (per wavefront of 4
topics: the slowest topic's) and loads per topic over a dict trie of the bench's own workload.

    python tools/walk_sim.py --subs 2000000 --topics 20000 [--window 4]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))


def build(w):
    from mqmatch import workload as W
    root = {}
    for f in W.strings(w["bytes"], w["offs"]):
        segs = f.split("/")
        if segs[0].lower() == "$share":
            segs = segs[2:]
        n = root
        for s in segs:
            n = n.setdefault(s, {})
    return root


def frontier(root, t):
    """k_walkf: rounds = levels; loads = literal probes + '+' child walk records."""
    L = len(t)
    front = [root]
    probes = loads = 0
    for d in range(L):
        nxt = []
        for n in front:
            probes += 1
            c = n.get(t[d])
            if d + 1 < L:
                if c is not None:
                    nxt.append(c)
                p = n.get("+")
                if p is not None:
                    loads += 1
                    nxt.append(p)
        front = nxt
        if not front:
            return d + 1, probes + loads
    return L, probes + loads


def prefix(root, t, window):
    """Prefix-hash walk: a branch (particle, depth) probes its literal continuation at up to
    `window` levels at once (one round), then spawns a branch per '+' child found on the way; a
    branch rooted at a '+' child also loads that child's walk record in its first round."""
    L = len(t)
    queue = [(root, 0, True)]  # (node, depth, needs walk record)
    rounds = probes = loads = 0
    while queue:
        rounds += 1
        nxt = []
        for n, d, wl in queue:
            loads += 1 if wl else 0
            chain = [(n, d)]
            m = min(L, d + window)
            probes += m - d
            x = n
            for j in range(d, m):
                x = x.get(t[j]) if x is not None else None
                if x is None:
                    break
                chain.append((x, j + 1))
            for node, depth in chain[0 if wl else 1:]:  # (a continuation's root spawned its '+' already)
                p = node.get("+")
                if p is not None and depth + 1 < L:
                    nxt.append((p, depth + 1, True))
            last, ld = chain[-1]
            if ld == m and m < L:  # the window ended inside an intact chain: continue it
                nxt.append((last, ld, False))
        queue = nxt
    return rounds, probes + loads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subs", type=int, default=2_000_000)
    ap.add_argument("--topics", type=int, default=20_000)
    ap.add_argument("--window", type=int, nargs="*", default=[16, 8, 4, 3])
    ap.add_argument("--mix", choices=["mqtt", "iot"], default="mqtt")
    args = ap.parse_args()
    from mqmatch import workload as W
    mix = W.MIX_IOT if args.mix == "iot" else W.MIX_MQTT
    w = W.gen_subscriptions(args.subs, max(1, args.subs // 10), seed=W.BASE_SEED, mix=mix)
    root = build(w)
    tb, to = W.gen_topics(w, args.topics, seed=W.BASE_SEED, mix=mix)
    topics = [s.split("/") for s in W.strings(tb, to)]
    res = {"frontier": [frontier(root, t) for t in topics]}
    for win in args.window:
        res[f"prefix w{win}"] = [prefix(root, t, win) for t in topics]
    n = len(topics)
    for k, v in res.items():
        rounds = sum(r for r, _ in v) / n
        wave = sum(max(r for r, _ in v[i:i + 4]) for i in range(0, n, 4)) / ((n + 3) // 4)
        loads = sum(x for _, x in v) / n
        print(f"{k:12s} rounds/topic {rounds:5.2f}  rounds/wave(4 topics) {wave:5.2f}  loads/topic {loads:6.2f}")


if __name__ == "__main__":
    main()
