"""Development helper: build one index, then time match_device under several knob settings
(env vars read by the engine per batch), interleaved and repeated to expose run-to-run noise.

  python tools/tune.py --subs 10000000 --steps 10 --repeat 2 \
      --configs "MQ_COPY_BLOCKS_PER_CU=8 MQ_MERGE_BLOCKS_PER_CU=8; MQ_COPY_BLOCKS_PER_CU=6"
"""
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
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--configs", default="")
    args = ap.parse_args()
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W

    torch.cuda.set_device(0)
    w = W.gen_subscriptions(args.subs, max(1, args.subs // 10), seed=W.BASE_SEED)
    eng = E.Engine(device=0, expected_subs=args.subs)
    eng.subscribe_bulk(w)
    from mqmatch import dist as D
    tb, to = W.gen_topics(w, args.topics, seed=D.topic_seed(0))  # bench.py's rank-0 batch
    n = len(to) - 1
    stream = torch.cuda.current_stream()
    d_tb = torch.from_numpy(tb).to("cuda:0")
    d_to = torch.from_numpy(to.view(np.int64)).to("cuda:0")
    eng.sync(stream.cuda_stream)
    configs = [c.strip() for c in args.configs.split(";")] if args.configs else [""]
    base_env = dict(os.environ)
    for rep in range(args.repeat):
        for cfg in configs:
            os.environ.clear()
            os.environ.update(base_env)
            for kv in cfg.split():
                k, v = kv.split("=", 1)
                os.environ[k] = v
            for _ in range(2):
                eng.match_device(d_tb.data_ptr(), d_to.data_ptr(), n, stream.cuda_stream)
            torch.cuda.synchronize()
            eng.profile(True)
            eng.profile_reset()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.match_device(d_tb.data_ptr(), d_to.data_ptr(), n, stream.cuda_stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            prof = eng.profile_read()
            eng.profile(False)
            ker = {k: round(v[1] / args.steps, 2) for k, v in prof.items() if v[1] > 0}
            print(json.dumps({"rep": rep, "config": cfg, "ms_per_step": round(dt * 1e3, 2),
                              "publishes_per_s_M": round(n / dt / 1e6, 2), "kernels_ms": ker}), flush=True)


if __name__ == "__main__":
    main()
