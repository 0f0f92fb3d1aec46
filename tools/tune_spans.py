"""Tuning harness for the span format: one index, several engine option settings timed
interleaved (mq_match_spans_device steps of a resident batch), one JSON line per (setting, rep).

  python tools/tune_spans.py --subs 10000000 --configs "7=1;7=6;7=8"

A config is ';'-separated; each is ','-separated option=value pairs (MQ_OPT_* numbers)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subs", type=int, default=10_000_000)
    ap.add_argument("--topics", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--configs", default="7=1;7=6;7=8")
    ap.add_argument("--work", action="store_true", help="also one step with MQ_PROF_WORK counters")
    ap.add_argument("--sort", action="store_true", help="experiment: the batch's topics sorted (byte order) on the host")
    args = ap.parse_args()
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(args.subs, max(1, args.subs // 10))
    eng = E.Engine()
    eng.subscribe_bulk(w)
    tb, to = W.gen_topics(w, args.topics)
    n = len(to) - 1
    if args.sort:  # locality experiment: topics that share a prefix walk together
        ts = sorted(bytes(tb[int(to[i]):int(to[i + 1])]) for i in range(n))
        to = np.zeros(n + 1, np.uint64)
        to[1:] = np.cumsum([len(t) for t in ts])
        tb = np.frombuffer(b"".join(ts) + bytes(16), np.uint8).copy()
    d_tb = torch.from_numpy(tb).cuda()
    d_to = torch.from_numpy(to.view(np.int64)).cuda()
    s = torch.cuda.current_stream()
    configs = [c.strip() for c in args.configs.split(";") if c.strip()]
    for rep in range(args.reps):
        for c in configs:
            for kv in c.split(","):
                k, v = kv.split("=")
                eng.set_option(int(k), int(v))
            for _ in range(2):
                eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, s.cuda_stream)
            eng.profile(True)
            eng.profile_reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, s.cuda_stream)
            torch.cuda.synchronize()
            ms = 1000 * (time.perf_counter() - t0) / args.steps
            prof = eng.profile_read()
            eng.profile(False)
            if args.work and rep == 0:
                eng.profile(True, work=True)
                eng.profile_reset()
                eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, s.cuda_stream)
                w = eng.profile_read()
                eng.profile(False)
                print(json.dumps({"config": c, "work": {k: v[0] for k, v in w.items() if v[1] == 0}}), flush=True)
            print(json.dumps({"config": c, "rep": rep, "subs": args.subs, "ms_per_step": ms,
                              "kernels_ms": {k: v[1] / args.steps for k, v in prof.items() if v[1] > 0},
                              "counters": {k: v[0] / args.steps for k, v in prof.items() if v[1] == 0}}),
                  flush=True)


if __name__ == "__main__":
    main()
