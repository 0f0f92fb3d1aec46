"""Tiny cases of the frontier walk by path hash against the oracle (windows 1 and 2): prints the
subscribers that differ."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("mqtt-server_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))


def main():
    from adapters import EngineAdapter, OracleAdapter
    from mqmatch import engine as E
    filters = ["#", "a/#", "a/b/#", "a/b/c/#", "a/b/c", "a/b", "a", "+/b/c", "a/+/c", "a/b/+", "+/+/+", "+/#",
               "a/+/#", "+/b/#", "a/b/c/d", "a/b/c/d/#", "a/b/c/+", "+/+/c/d"]
    topics = ["a", "a/b", "a/b/c", "a/b/c/d", "a/b/c/d/e", "x/b/c", "a/x/c", "a/b/x", "x/y/z", "x/b/c/d"]
    for win in (1, 2, 3):
        e, o = EngineAdapter(), OracleAdapter()
        e.x.engine.set_option(E.OPT_WALK_WINDOW, win)
        for k, f in enumerate(filters):
            e.subscribe(f"c{k}", f)
            o.subscribe(f"c{k}", f)
        for t, g in zip(topics, e.subscribers_batch(topics)):
            want = o.subscribers(t)
            if g != want:
                gs, ws = set(g["subscriptions"]), set(want["subscriptions"])
                print(f"win {win} topic {t}: missing {sorted(ws - gs)} extra {sorted(gs - ws)}", flush=True)
                for c in sorted(ws - gs):
                    print("    missing", c, filters[int(c[1:])])
        print(f"win {win} done", flush=True)


if __name__ == "__main__":
    main()
