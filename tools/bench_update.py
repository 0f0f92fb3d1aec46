"""Update-path measurement: how fast the index is built and
kept current, beside the match path bench.py measures.

  build     mq_subscribe_bulk on an empty index (the restore path, server.go:1624-1640) vs the
            per-entry path (the same call on a non-empty index: one mq_subscribe per entry)
            over a sample; then the first mq_sync (whole image upload).
  churn     K random live subscriptions unsubscribed (mq_unsubscribe, one ctypes call each —
            the call overhead is measured and reported beside) and K new ones subscribed
            (mq_subscribe_bulk on the non-empty index: the per-entry C loop, no Python per
            entry); then mq_sync: its latency and upload bytes (dirty 64 KiB pages only).
            After the last batch one span-format match step checks the image still matches.
  retained  mq_retain_bulk of N retained topics (loadRetained, server.go:1688-1692) vs the
            per-entry path over a sample.

Prints one JSON object. Run on the GPU box (mq_sync and the match need the device):
  python tools/bench_update.py --subs 10000000 --retained 100000000
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mqtt-server_amd"))
from mqmatch import engine as E  # noqa: E402
from mqmatch import workload as W  # noqa: E402


def _slice(w, lo, hi):
    o = w["offs"][lo:hi + 1]
    return {"bytes": w["bytes"][int(o[0]):int(o[-1])].copy() if int(o[-1]) > int(o[0]) else np.zeros(1, np.uint8),
            "offs": (o - o[0]).astype(np.uint64),
            **{k: w[k][lo:hi] for k in ("client_ids", "filter_ids", "qos", "flags", "idents")}}


def _sync(e, torch):
    if not torch.cuda.is_available():  # a CPU dry run of the host side
        return None, None
    s0 = e.stats()
    torch.cuda.synchronize()
    t = time.perf_counter()
    e.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    s1 = e.stats()
    return dt * 1e3, s1["upload_bytes_total"] - s0["upload_bytes_total"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subs", type=int, default=10_000_000)
    ap.add_argument("--clients", type=int, default=0, help="default subs/10")
    ap.add_argument("--per-entry-sample", type=int, default=0, help="default: every entry")
    ap.add_argument("--churn", default="1000,10000,100000,1000000")
    ap.add_argument("--retained", type=int, default=0)
    ap.add_argument("--retained-sample", type=int, default=2_000_000)
    ap.add_argument("--topics", type=int, default=1_000_000)
    a = ap.parse_args()
    t0 = time.time()

    def beat():  # a progress line every 30 s (long builds print nothing otherwise)
        while True:
            time.sleep(30)
            print(f"[bench_update] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    import torch
    out = {"subs": a.subs}
    L = E.lib()

    w = W.gen_subscriptions(a.subs, a.clients or max(1, a.subs // 10))
    n = len(w["client_ids"])
    # build: bulk vs per-entry (sample)
    t = time.perf_counter()
    e = E.Engine()
    e.subscribe_bulk(w)
    tb = time.perf_counter() - t
    m = min(a.per_entry_sample or n, n)
    p = E.Engine()
    p.subscribe_bulk(_slice(w, 0, 1))
    t = time.perf_counter()
    p.subscribe_bulk(_slice(w, 1, m))
    tp = time.perf_counter() - t
    p.close()
    out["build"] = {"bulk_s": tb, "bulk_subs_per_s": n / tb, "per_entry_sample": m,
                    "per_entry_subs_per_s": (m - 1) / tp, "speedup": (n / tb) / ((m - 1) / tp),
                    "threads": min(16, os.cpu_count() or 1)}
    ms, nb = _sync(e, torch)
    out["build"]["first_sync_ms"], out["build"]["first_sync_bytes"] = ms, nb
    st = e.stats()
    out["build"]["image"] = {k: st[k] for k in ("nodes", "edges", "subs", "subs_merge", "shared", "partners",
                                                "device_bytes")}

    # churn
    raw = w["bytes"].tobytes()
    offs = w["offs"]
    rng = np.random.default_rng(7)
    unsub = L.mq_unsubscribe
    t = time.perf_counter()
    for _ in range(100_000):
        L.mq_retained_len(e.h)
    call_ns = (time.perf_counter() - t) / 100_000 * 1e9
    churn = []
    next_client = int(w["client_ids"].max()) + 1
    step = None
    if torch.cuda.is_available():
        # one span-format match step of a fixed batch, clean and after each churn round (the
        # image is updated in place: probe chains, pair lists and slabs must not degrade)
        tb_, to_ = W.gen_topics(w, a.topics)
        d_b = torch.from_numpy(tb_).cuda()
        d_o = torch.from_numpy(to_.view(np.int64)).cuda()

        def step(reps=5):
            e.match_spans_device(d_b.data_ptr(), d_o.data_ptr(), len(to_) - 1)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(reps):
                e.match_spans_device(d_b.data_ptr(), d_o.data_ptr(), len(to_) - 1)
            torch.cuda.synchronize()
            return (time.perf_counter() - t) / reps * 1e3
        out["match_clean_ms_per_step"] = step()
    for k in (int(x) for x in a.churn.split(",") if x):
        k = min(k, n // 2)
        idx = rng.choice(n, k, replace=False)
        fs = [raw[int(offs[i]):int(offs[i + 1])] for i in idx]
        cs = w["client_ids"][idx].tolist()
        # the first half one ctypes call each (mq_unsubscribe), the second half in one
        # mq_unsubscribe_bulk call
        h = k // 2
        t = time.perf_counter()
        removed = 0
        for f, c in zip(fs[:h], cs[:h]):
            removed += unsub(e.h, f, len(f), c) == 1
        tu = time.perf_counter() - t
        ub = np.frombuffer(b"".join(fs[h:]) or b"\0", np.uint8).copy()
        uo = np.zeros(k - h + 1, np.uint64)
        uo[1:] = np.cumsum([len(f) for f in fs[h:]])
        t = time.perf_counter()
        removed += int(e.unsubscribe_bulk(ub, uo, np.array(cs[h:], np.uint32)).sum())
        tub = time.perf_counter() - t
        sel = np.sort(idx)
        bs = [raw[int(offs[i]):int(offs[i + 1])] for i in sel]
        no = np.zeros(k + 1, np.uint64)
        no[1:] = np.cumsum([len(b) for b in bs])
        ins = {"bytes": np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy(), "offs": no,
               "client_ids": (next_client + np.arange(k)).astype(np.uint32), "filter_ids": w["filter_ids"][sel],
               "qos": w["qos"][sel], "flags": w["flags"][sel], "idents": w["idents"][sel]}
        next_client += k
        t = time.perf_counter()
        e.subscribe_bulk(ins)
        ts = time.perf_counter() - t
        ms, nb = _sync(e, torch)
        churn.append({"ops": k, "unsubscribed": int(removed),
                      "unsubscribe_per_s": h / max(tu, 1e-9), "unsubscribe_per_s_less_call": h / max(1e-9, tu - h * call_ns * 1e-9),
                      "unsubscribe_bulk_per_s": (k - h) / max(tub, 1e-9), "subscribe_per_s": k / ts, "sync_ms": ms, "sync_bytes": nb,
                      "sync_bytes_per_op": None if nb is None else nb / (2 * k),
                      "match_ms_per_step": step() if step else None})
    out["churn"] = churn
    out["ctypes_call_ns"] = call_ns
    e.check()
    if step:
        out["match_after_churn_ms_per_step"] = churn[-1]["match_ms_per_step"] if churn else step()
    e.close()
    del w

    if a.retained:
        rb, ro, hd, _ = W.gen_retained(a.retained, n_sys=1000)
        t = time.perf_counter()
        r = E.Engine()
        r.retain_bulk(rb, ro, hd)
        trb = time.perf_counter() - t
        rl = r.retained_len()
        r.close()
        m = min(a.retained_sample, a.retained)
        q = E.Engine()
        q.retain_bulk(rb, ro[:2] - ro[0], hd[:1])
        t = time.perf_counter()
        q.retain_bulk(rb[int(ro[1]):int(ro[m])], (ro[1:m + 1] - ro[1]).astype(np.uint64), hd[1:m])
        trp = time.perf_counter() - t
        q.close()
        out["retained"] = {"n": a.retained, "live": rl, "bulk_s": trb, "bulk_per_s": a.retained / trb,
                           "per_entry_sample": m, "per_entry_per_s": (m - 1) / trp,
                           "speedup": (a.retained / trb) / ((m - 1) / trp)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
