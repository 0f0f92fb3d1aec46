"""End-to-end probe: mq_match_spans (host topics in, host span results out) on bench.py's index and
batch, timed per call, for a rocprofv3 kernel + memory-copy trace of where the time goes.

  rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/e2e -- python3 tools/e2e_probe.py
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subs", type=int, default=10_000_000)
    ap.add_argument("--topics", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from mqmatch import engine as E
    from mqmatch import workload as W
    w = W.gen_subscriptions(args.subs, max(1, args.subs // 10), seed=W.BASE_SEED)
    eng = E.Engine(expected_subs=args.subs)
    eng.subscribe_bulk(w)
    tb, to = W.gen_topics(w, args.topics, seed=W.BASE_SEED)
    n = len(to) - 1
    eng.match_spans_host(tb, to)
    for rep in range(args.reps):
        t0 = time.perf_counter()
        nbytes, _ = eng.match_spans_host(tb, to)
        dt = time.perf_counter() - t0
        print(json.dumps({"rep": rep, "topics": n, "ms": 1e3 * dt, "publishes_per_s": n / dt,
                          "result_bytes": nbytes, "topic_bytes": int(to[-1]),
                          "bytes_per_topic": {k: v / n for k, v in eng.last_host_bytes.items()}}), flush=True)


if __name__ == "__main__":
    main()
