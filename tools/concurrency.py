"""Do two batches in flight on one GPU beat one? The 10M config-3 index of bench.py built into K
engine handles (K copies of the image in HBM), each matching its own 1M-topic batch
(mq_match_spans_device, device results) on its own host thread and stream, back to back for
--steps steps: aggregate publishes/s against one handle alone. A measurement of the device's
headroom for overlapping batches, not a product path.

  python tools/concurrency.py --handles 2 [--subs 10000000] [--topics 1000000] [--steps 20]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--handles", type=int, default=2)
    ap.add_argument("--subs", type=int, default=10_000_000)
    ap.add_argument("--topics", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(args.subs, max(1, args.subs // 10), seed=W.BASE_SEED)
    engs, batches = [], []
    for k in range(args.handles):
        e = E.Engine(device=0, expected_subs=args.subs)
        e.subscribe_bulk(w)
        tb, to = W.gen_topics(w, args.topics, seed=W.BASE_SEED + 1000 * k)
        d_tb = torch.from_numpy(tb).cuda()
        d_to = torch.from_numpy(to.view(np.int64)).cuda()
        s = torch.cuda.Stream()
        e.sync(s.cuda_stream)
        engs.append(e)
        batches.append((d_tb, d_to, len(to) - 1, s))
    torch.cuda.synchronize()

    def run(k, steps):
        d_tb, d_to, n, s = batches[k]
        for _ in range(steps):
            engs[k].match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, s.cuda_stream)

    for k in range(args.handles):  # walk trials, buffer sizing
        run(k, 10)
    torch.cuda.synchronize()
    out = {"subs": args.subs, "topics_per_batch": args.topics, "steps": args.steps}
    t0 = time.perf_counter()
    run(0, args.steps)
    torch.cuda.synchronize()
    one = time.perf_counter() - t0
    out["one_handle"] = {"publishes_per_s": args.topics * args.steps / one, "ms_per_step": 1e3 * one / args.steps}
    th = [threading.Thread(target=run, args=(k, args.steps)) for k in range(args.handles)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    many = time.perf_counter() - t0
    out[f"{args.handles}_handles"] = {"publishes_per_s": args.handles * args.topics * args.steps / many,
                                      "ms_per_step_each": 1e3 * many / args.steps}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
