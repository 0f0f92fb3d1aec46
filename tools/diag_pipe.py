"""Diagnosis (GPU): an update between two pipelined submits — which results differ from the oracle."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mqtt-server_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle as O  # noqa: E402
from digest import engine_digests  # noqa: E402
from mqmatch import engine as E  # noqa: E402
from mqmatch import workload as W  # noqa: E402

w = W.gen_subscriptions(40000, 3000, seed=73)
eng, orc = E.Engine(), O.OracleIndex()
assert (eng.subscribe_bulk(w) == orc.subscribe_bulk(w)).all()
tb, to = W.gen_topics(w, 2000, seed=90)


def submit():
    t = C.c_void_p()
    assert E.lib().mq_match_spans_submit(eng.h, E._p(tb, E._u8p), E._p(to, E._u64p), 2000, C.byref(t)) == 0
    return t


def wait(t):
    rp = C.POINTER(E.SpanResult)()
    assert E.lib().mq_match_spans_wait(t, C.byref(rp)) == 0
    return E._expand_host_spans(rp, 2000)


mode = sys.argv[1] if len(sys.argv) > 1 else "held"
before = orc.digest_batch(tb, to, nthreads=8)[0]
t0 = submit() if mode == "held" else None
print("sub", eng.subscribe("#", 999999, 777, 2, 0, 0), orc.subscribe("c999999", "#", qos=2, client_id=999999, filter_id=777))
after = orc.digest_batch(tb, to, nthreads=8)[0]
try:
    eng.check()
    print("host check ok")
except Exception as e:
    print("host check FAILED", e)
try:
    eng.device_check()
    print("device check ok")
except Exception as e:
    print("device check FAILED", e)
t1 = submit()
if t0 is not None:
    print("t0 vs before: bad", int((engine_digests(wait(t0))[0] != before).sum()))
print("t1 vs after: bad", int((engine_digests(wait(t1))[0] != after).sum()), "of", len(after))
print("sync spans vs after: bad", int((engine_digests(eng.match_batch_spans(tb, to))[0] != after).sum()))
print("rows vs after: bad", int((engine_digests(eng.match_batch(tb, to))[0] != after).sum()))
