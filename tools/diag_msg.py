"""Diagnostic: build N retained topics (config 5 generator), check the host image
(mq_index_check), then one Messages batch through the level-order image.
  python tools/diag_msg.py 100000000"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mqtt-server_amd"))
from mqmatch import engine as E  # noqa: E402
from mqmatch import workload as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
t = time.time()


def _beat():  # a line every 30 s: long host phases are not a hung run
    while True:
        time.sleep(30)
        print(f"... working ({time.time() - t:.0f}s)", flush=True)


threading.Thread(target=_beat, daemon=True).start()
rb, ro, hd, rh = W.gen_retained(n, n_sys=1000, seed=W.BASE_SEED + 3)
fb, fo = W.gen_msg_filters(rh, 1000, seed=W.BASE_SEED + 4)
print("generated", n, round(time.time() - t, 1), flush=True)
e = E.Engine(device=0)
e.retain_bulk(rb, ro, hd)
print("built", round(time.time() - t, 1), e.stats(), flush=True)
if "--check" in sys.argv:
    e.check()
    print("host check ok", round(time.time() - t, 1), flush=True)
try:
    e.device_check()
    print("device check ok", round(time.time() - t, 1), flush=True)
except Exception as ex:
    print("device check FAILED:", ex, flush=True)
for img in (1, 0):
    e.set_option(E.OPT_MSG_IMAGE, img)
    try:
        base, count, hs = e.messages_batch(fb, fo)
        print("messages image" if img else "messages walk", "ok: handles", int(count.sum()), flush=True)
    except Exception as ex:
        print("messages image" if img else "messages walk", "FAILED:", ex, flush=True)
