"""Diagnosis (GPU): where a pipelined host-result batch spends its time — the submit call (upload,
kernels, packing) and the wait (the copy's remainder) — for consecutive 1M-topic batches at 10M
subscriptions; optional pinned topic buffers."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mqtt-server_amd")]
from mqmatch import engine as E  # noqa: E402
from mqmatch import workload as W  # noqa: E402

subs = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
if "--torch" in sys.argv:  # as bench.py: torch's HIP runtime up first, a tensor on the device
    import torch
    _keep = torch.zeros(1 << 20, device="cuda")
w = W.gen_subscriptions(subs, subs // 10)
eng = E.Engine(expected_subs=subs if "--expected" in sys.argv else 0)
eng.subscribe_bulk(w)
tb, to = W.gen_topics(w, 1_000_000)
n = len(to) - 1
pinned = "--pinned" in sys.argv
if pinned:
    import torch
    tbp = torch.empty(len(tb), dtype=torch.uint8).pin_memory()
    tbp.numpy()[:] = tb
    top = torch.empty(len(to), dtype=torch.int64).pin_memory()
    top.numpy()[:] = to.view(np.int64)
    tb, to = tbp.numpy(), top.numpy().view(np.uint64)


def submit():
    t = C.c_void_p()
    E._check(E.lib().mq_match_spans_submit(eng.h, E._p(tb, E._u8p), E._p(to, E._u64p), n, C.byref(t)), "submit")
    return t


def wait(t):
    rp = C.POINTER(E.SpanResult)()
    E._check(E.lib().mq_match_spans_wait(t, C.byref(rp)), "wait")
    E.lib().mq_result_free(rp)


for _ in range(2):
    wait(submit())
if "--seq-first" in sys.argv:  # as bench.py: plain host-result calls before the pipelined ones
    for _ in range(4):
        eng.match_spans_host(tb, to)
log = []
t0 = time.perf_counter()
pend = []
for k in range(6):
    a = time.perf_counter()
    pend.append(submit())
    b = time.perf_counter()
    if len(pend) == 2:
        wait(pend.pop(0))
    c = time.perf_counter()
    log.append({"k": k, "submit_ms": round(1e3 * (b - a), 3), "wait_prev_ms": round(1e3 * (c - b), 3)})
while pend:
    wait(pend.pop(0))
dt = time.perf_counter() - t0
print(json.dumps({"argv": sys.argv[1:], "pinned": pinned, "batches": 6, "ms_per_batch": 1e3 * dt / 6, "publishes_per_s": 6 * n / dt,
                  "steps": log}))
t = time.perf_counter()
for _ in range(3):
    a = time.perf_counter()
    wait(submit())
print(json.dumps({"sequential_ms_per_batch": 1e3 * (time.perf_counter() - t) / 3}))
