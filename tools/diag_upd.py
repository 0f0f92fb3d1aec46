"""Diagnosis (GPU): one subscribe after a bulk load, checked against the oracle, for several
(client id, filter id) choices."""
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
tb, to = W.gen_topics(w, 2000, seed=90)
nf = int(w["filter_ids"].max()) + 1
for cid, fid, filt, qos in [(999999, 777, "#", 2), (999999, nf, "#", 2), (3001, nf + 1, "#", 2), (999999, nf, "#", 0),
                            (999999, nf, "zz/+", 2)]:
    eng, orc = E.Engine(), O.OracleIndex()
    assert (eng.subscribe_bulk(w) == orc.subscribe_bulk(w)).all()
    b0 = int((engine_digests(eng.match_batch_spans(tb, to))[0] != orc.digest_batch(tb, to, nthreads=8)[0]).sum())
    r = (eng.subscribe(filt, cid, fid, qos, 0, 0), orc.subscribe("c%d" % cid, filt, qos=qos, client_id=cid, filter_id=fid))
    od, ocnt, _ = orc.digest_batch(tb, to, nthreads=8)
    dg, cnt = engine_digests(eng.match_batch_spans(tb, to))
    bad = np.nonzero(dg != od)[0]
    print(cid, fid, filt, qos, "answers", r, "bad before", b0, "after", len(bad),
          "first counts", cnt[bad[:2]].tolist() if len(bad) else None, ocnt[bad[:2]].tolist() if len(bad) else None)
    eng.close()
