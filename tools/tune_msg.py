"""Development helper: build one retained index, then time Messages batches under several
MQ_MSG_WPE / MQ_MSG_SPEC_MB settings (read by the engine per batch), interleaved to expose
run-to-run noise. python tools/tune_msg.py --retained 10000000 --configs "1;6;8" """
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
    ap.add_argument("--retained", type=int, default=10_000_000)
    ap.add_argument("--filters", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--configs", default="1;6;8", help="MQ_MSG_WPE values, ';'-separated")
    args = ap.parse_args()
    import torch
    from mqmatch import engine as E
    from mqmatch import workload as W
    rb, ro, hd, rh = W.gen_retained(args.retained, n_sys=1000, seed=W.BASE_SEED + 3)
    fb, fo = W.gen_msg_filters(rh, args.filters, seed=W.BASE_SEED + 4)
    n = len(fo) - 1
    eng = E.Engine(device=0)
    eng.retain_bulk(rb, ro, hd)
    s = torch.cuda.current_stream()
    d_fb = torch.from_numpy(np.concatenate([fb, np.zeros(16, np.uint8)])).cuda()
    d_fo = torch.from_numpy(fo.view(np.int64)).cuda()
    res = {}
    for rep in range(args.repeat):
        for c in args.configs.split(";"):
            os.environ["MQ_MSG_WPE"] = c.strip()
            eng.messages_device(d_fb.data_ptr(), d_fo.data_ptr(), n, s.cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.messages_device(d_fb.data_ptr(), d_fo.data_ptr(), n, s.cuda_stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            res.setdefault(c.strip(), []).append(ms)
            print(json.dumps({"MQ_MSG_WPE": c.strip(), "rep": rep, "ms_per_step": ms}), flush=True)
    print(json.dumps({k: min(v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
