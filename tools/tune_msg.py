"""Development helper: build one retained index, then time Messages batches under several
engine option settings (`opt=value` pairs, ','-separated; configs ';'-separated), interleaved to
expose run-to-run noise; --work adds one step with the count pass's per-filter clocks and fan-out
counters (MQ_PROF_WORK). python tools/tune_msg.py --retained 10000000 --configs "3=64;3=0" --work"""
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
    ap.add_argument("--configs", default="3=64", help="option=value pairs (',') per config (';')")
    ap.add_argument("--work", action="store_true")
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
            for kv in c.split(","):
                if kv.strip():
                    k, v = kv.split("=")
                    eng.set_option(int(k), int(v))
            eng.messages_device(d_fb.data_ptr(), d_fo.data_ptr(), n, s.cuda_stream)
            torch.cuda.synchronize()
            eng.profile(True)
            eng.profile_reset()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.messages_device(d_fb.data_ptr(), d_fo.data_ptr(), n, s.cuda_stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            prof = eng.profile_read()
            eng.profile(False)
            res.setdefault(c.strip(), []).append(ms)
            out = {"config": c.strip(), "rep": rep, "ms_per_step": ms,
                   "kernels_ms": {k: v[1] / args.steps for k, v in prof.items() if v[1] > 0}}
            if args.work and rep == 0:
                eng.profile(True, work=True)
                eng.profile_reset()
                eng.messages_device(d_fb.data_ptr(), d_fo.data_ptr(), n, s.cuda_stream)
                torch.cuda.synchronize()
                w = eng.profile_read()
                eng.profile(False)
                out["work"] = {k: v[0] for k, v in w.items() if v[1] == 0}
            print(json.dumps(out), flush=True)
    print(json.dumps({k: min(v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
