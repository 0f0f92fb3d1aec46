"""A/B of engine options on one index and one batch, in one process (no box-to-box noise): the
10M config-3 index of bench.py and its rank-0 1M-topic batch; each variant (a list of
MQ_OPT=value settings) runs --steps device steps with kernel timing, the variants in turn, for
--rounds rounds; per variant the median per-step kernel times, and one step's results digested
per topic (a cheap order-free checksum of every topic's expanded rows) equal across variants.

  python tools/ab_options.py --variants "18=0" "18=512" [--subs 10000000] [--topics 1000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def log(msg):
    print(f"[ab {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--subs", type=int, default=10_000_000)
    ap.add_argument("--topics", type=int, default=1_000_000)
    ap.add_argument("--mix", choices=["mqtt", "iot"], default="mqtt")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--check", type=int, default=20000, help="topics whose expanded rows are compared across variants")
    args = ap.parse_args()
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    from digest import engine_digests
    mix = W.MIX_IOT if args.mix == "iot" else W.MIX_MQTT
    clients = args.subs if args.mix == "iot" else max(1, args.subs // 10)
    w = W.gen_subscriptions(args.subs, clients, seed=W.BASE_SEED, mix=mix)
    eng = E.Engine(device=0, expected_subs=args.subs)
    eng.subscribe_bulk(w)
    tb, to = W.gen_topics(w, args.topics, seed=W.BASE_SEED, mix=mix)
    n = len(to) - 1
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    eng.sync(None)
    torch.cuda.synchronize()
    log(f"index {eng.stats()}")

    def setv(v):
        for kv in v.split(","):
            k, x = kv.split("=")
            eng.set_option(int(k), int(x))

    def step():
        return eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, None)

    for _ in range(10):  # walk trials and buffer sizing, outside the comparison
        step()
    torch.cuda.synchronize()
    times = {v: [] for v in args.variants}
    digests = {}
    for rnd in range(args.rounds):
        for v in args.variants:
            setv(v)
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            eng.profile(True)
            eng.profile_reset()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                r = step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            prof = eng.profile_read()
            eng.profile(False)
            times[v].append({"step_ms": 1e3 * dt / args.steps,
                             **{k: p[1] / args.steps for k, p in prof.items() if p[1] > 0}})
            if rnd == 0 and args.check:
                dg, _ = engine_digests(E.expand_device_spans(r, n, args.check))
                digests[v] = dg
            log(f"round {rnd} {v}: {times[v][-1]}")
    base = args.variants[0]
    out = {"subs": args.subs, "topics": n, "steps": args.steps, "rounds": args.rounds, "variants": {}}
    for v in args.variants:
        keys = sorted(set().union(*[t.keys() for t in times[v]]))
        out["variants"][v] = {k: float(np.median([t.get(k, 0.0) for t in times[v]])) for k in keys}
        if args.check:
            out["variants"][v]["results_equal_to_" + base] = bool((digests[v] == digests[base]).all())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
