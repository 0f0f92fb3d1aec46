"""Diagnosis: distribution of shared rows per topic (what k_pick walks) on the bench workload."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
from mqmatch import engine as E  # noqa: E402
from mqmatch import workload as W  # noqa: E402

subs = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
w = W.gen_subscriptions(subs, max(1, subs // 10), seed=W.BASE_SEED, mix=W.MIX_MQTT)
eng = E.Engine(expected_subs=subs)
eng.subscribe_bulk(w)
tb, to = W.gen_topics(w, 20000, seed=W.BASE_SEED + 2, mix=W.MIX_MQTT)
r = eng.match_batch(tb, to)
ns = r["n_shared"].astype(np.int64)
nf = []
for t in range(len(ns)):
    b = int(r["shared_base"][t])
    nf.append(len(np.unique(r["shared"][b:b + ns[t], 0])))
nf = np.array(nf)
print("topics", len(ns), "shared rows/topic mean", ns.mean(), "max", ns.max(),
      "p50/p90/p99", np.percentile(ns, [50, 90, 99]), "zero-share topics", (ns == 0).mean())
print("distinct shared filters/topic mean", nf.mean(), "max", nf.max(), "p99", np.percentile(nf, 99))
print("rows per topic (all)", (r["sub_cap"].astype(np.int64)).mean())
