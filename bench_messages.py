"""Secondary benchmark: the retained-message reverse match (Messages, topics.go:525-579) —
BASELINE.json config 5 ("100M retained topics x 100k wildcard subscribe filters"), scaled by
--retained (default 10M retained topics, 10 % of config 5; the 100M-topic host image does not
fit the build container). A step is one Messages batch of --filters filters already in HBM:
--format runs (the default, round 6): mq_messages_runs_device — the walk over the level-order
retained image (k_msgq count pass, scan, place pass) leaves each filter's result as runs of the
image's handle array, as SURVEY.md §7 step 8 plans ("expanded at the boundary"); --format
handles: mq_messages_device, the same walk plus k_msg_copy writing every handle.

Prints one JSON line like bench.py's: throughput, output handles per filter, the k_msg roofline
(algorithmic bytes B = 8·L + 4 + 16·P + 16·O per filter, SURVEY.md §8d, from the oracle's exact
counters on a sample, over the two k_msg launches' HIP-event time) and the CPU baseline (the
oracle's Messages on 16 host threads over a bounded sample).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))
HBM_PEAK_GBS = 8000.0


def heartbeat(period=30.0):
    """Log a line every `period` s from a daemon thread, so that long host phases (generating or
    building a 50M-100M entry index) are not mistaken for a hung run."""
    import threading
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            log(f"... working ({time.time() - t0:.0f}s)")
    threading.Thread(target=run, daemon=True).start()


def log(msg):
    print(f"[bench_messages {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def read_msg_traffic(n_retained, n_filters, fmt="handles", key_index=True, export=1):
    """HBM bytes per Messages step (k_msgq passes + k_msg_copy: FETCH_SIZE x1 for the walks' random
    loads, x2 for k_msg_copy's streams, + WRITE_SIZE) from a committed rocprofv3 PMC summary of the
    same configuration (retained topics, filters per step, export threshold, output format), if
    present."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as f:
            e = json.load(f).get("messages" if fmt == "handles" else "messages_runs", {}).get(str(n_retained))
        if e is None or int(e["filters"]) != n_filters or int(e.get("export", 1)) != export:
            return None
        if bool(e.get("key_index", False)) != key_index:  # (the round-6 entries were taken with the key index)
            return None
        return float(e["hbm_bytes_per_step"])
    except (OSError, ValueError, KeyError, TypeError):
        return None


def handle_digests(base, count, hs):
    """Per-filter digest of the sorted handles, as the oracle's messages_digest_batch computes
    it (fold of the count, then of each handle in ascending order), vectorised over filters."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from digest import fold, SEED
    n = len(count)
    m = int(count.max()) if n else 0
    mat = np.zeros((n, max(m, 1)), np.uint64)
    for i in range(n):
        mat[i, :count[i]] = np.sort(hs[int(base[i]):int(base[i]) + int(count[i])])
    d = fold(np.full(n, SEED, np.uint64), count.astype(np.uint64))
    for k in range(m):
        live = count > k
        d = np.where(live, fold(d, mat[:, k]), d)
    return d


def oracle_side(rb, ro, hd, fb, fo, n, args, early=None):
    """The oracle's part of the bench: sample digests and counters (SURVEY.md §8d B terms) and
    the CPU baseline (the oracle's Messages on 16 host threads over a bounded sample). early(o):
    called with the parity part as soon as it exists (--oracle-only writes it before the CPU
    baselines are timed)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    t0 = time.time()
    orc = O.OracleIndex()
    orc.retain_bulk(rb, ro, hd)
    log(f"oracle index built in {time.time() - t0:.1f}s")
    ns = min(n, 4096)
    dg, cnt, tot = orc.messages_digest_batch(fb, fo[:ns + 1], nthreads=16)
    # the baseline: the fast restatement (oracle/topics_fast.h FastMsgIndex: flat nodes, handles
    # looked up at build time, segments split once; digest-equal to the oracle), 16 threads; the
    # literal restatement beside it
    t0 = time.time()
    fast = orc.fast_messages()
    log(f"fast CPU restatement built in {time.time() - t0:.1f}s")
    # every filter of the batch through the fast restatement, pinned to the oracle on the sample
    t0 = time.time()
    fdg, fcnt = fast.digest_batch(fb, fo, nthreads=16)
    pinned = bool((fdg[:ns] == dg).all() and (fcnt[:ns] == cnt).all())
    log(f"fast restatement digests of all {n} filters in {time.time() - t0:.1f}s; equal to the oracle's "
        f"on the {ns}-filter sample: {pinned}")
    if not pinned:
        raise SystemExit("the fast restatement differs from the oracle on the sample")
    o = {"sample_filters": ns, "digests": [format(int(x), "x") for x in dg], "counts": [int(x) for x in cnt],
         "all_digests": [format(int(x), "x") for x in fdg], "all_counts": [int(x) for x in fcnt],
         "all_note": "fast restatement (oracle/topics_fast.cpp), equal to the oracle on the sample",
         "per_filter": {k: v / ns for k, v in tot.items()}, "cpu": None}
    if early:
        early(o)
    cal = min(n, 2048)
    secs, _ = fast.bench_messages(fb, fo[:cal + 1], 16)
    m = int(min(n, max(cal, cal * args.cpu_seconds / max(secs, 1e-6))))
    log(f"CPU baseline: calibration {cal} filters in {secs:.2f}s; timing {m} filters")
    secs, _ = fast.bench_messages(fb, fo[:m + 1], 16)
    log(f"CPU baseline: {m} filters in {secs:.2f}s")
    cpu = {"value": m / secs, "unit": "filters/s", "cores": 16, "kind": "port",
           "sample": f"first {m} filters, 16 threads, Messages() per filter: the fast CPU restatement of the Go "
                     f"trie's scanMessages (oracle/topics_fast.cpp FastMsgIndex; digest-equal to the oracle)"}
    fast.close()
    del fast
    if len(ro) - 1 < 50_000_000:  # (the literal restatement beside it; at config 5's full size it is
        lcal = min(n, 512)        #  ~600 filters/s and holds ~120 GB: not timed)
        lsecs, _ = orc.bench_messages(fb, fo[:lcal + 1], 16)
        lm = int(min(n, max(lcal, lcal * min(5.0, args.cpu_seconds / 2) / max(lsecs, 1e-6))))
        lsecs, _ = orc.bench_messages(fb, fo[:lm + 1], 16)
        cpu["literal"] = {"value": lm / lsecs, "sample": f"first {lm} filters, 16 threads, oracle/topics_oracle.cpp"}
        log(f"literal CPU baseline: {lm} filters in {lsecs:.2f}s")
    o["cpu"] = cpu
    return o


def full_parity(eng, fb, fo, o, max_handles=150_000_000):
    """Every filter of the batch: the engine's Messages (mq_messages_batch, host results, in chunks
    of at most ~max_handles handles) digested per filter as the oracle digests its own
    (oracle/oracle_capi.cpp orc_handle_digests, the checker), against the --oracle-only side's
    fast-restatement digests of all filters."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    n = len(fo) - 1
    want = np.array([int(x, 16) for x in o["all_digests"]], np.uint64)
    wcnt = np.array(o["all_counts"], np.uint64)
    # chunk boundaries from the expected counts, so that no chunk's host result outgrows memory
    bounds, acc, a = [], 0, 0
    for i in range(n):
        acc += int(wcnt[i])
        if acc >= max_handles or i - a >= 16383:
            bounds.append((a, i + 1))
            a, acc = i + 1, 0
    if a < n:
        bounds.append((a, n))
    bad_d = bad_c = 0
    for a, b in bounds:
        sub_o = (fo[a:b + 1] - fo[a]).astype(np.uint64)
        sub_b = np.ascontiguousarray(fb[int(fo[a]):int(fo[b])])
        base, count, hs = eng.messages_batch(sub_b, sub_o)
        bad_c += int((count.astype(np.uint64) != wcnt[a:b]).sum())
        bad_d += int((O.handle_digests(base, count, hs, nthreads=16) != want[a:b]).sum())
        del base, count, hs
    return {"filters": n, "chunks": len(bounds), "counts_differ": bad_c, "digests_differ": bad_d,
            "digests_equal": bad_c == 0 and bad_d == 0,
            "against": o.get("all_note", "fast restatement")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--retained", type=int, default=10_000_000)
    ap.add_argument("--sys", type=int, default=1000, help="$SYS/... retained topics (Q4)")
    ap.add_argument("--filters", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--format", choices=["runs", "handles"], default="runs",
                    help="runs: mq_messages_runs_device (each filter's result as runs of the image's handles); "
                         "handles: mq_messages_device (every handle copied out)")
    ap.add_argument("--walk", action="store_true",
                    help="Messages by the particle walk (MQ_OPT_MSG_IMAGE 0) instead of the level-order image")
    ap.add_argument("--no-img-edges", action="store_true",
                    help="literal lookups through the index's edge table instead of the image's (MQ_OPT_MSG_EDGES 0)")
    ap.add_argument("--no-key-index", action="store_true",
                    help="a literal under wide runs probes each particle, without the image's key index "
                         "(MQ_OPT_MSG_KEYIDX 0)")
    ap.add_argument("--key-index-rounds", type=int, default=0,
                    help="MQ_OPT_MSG_KEYIDX N (N >= 2): a literal level tries the key index above N rounds "
                         "of particle probes instead of kKxMinRounds")
    ap.add_argument("--export", type=int, default=1,
                    help="MQ_OPT_MSG_EXPORT: 0 off, 1 kMsgExportMin (default), else the threshold (hits under the "
                         "key index, particles without it) above which a filter's literal level goes to work items")
    ap.add_argument("--oracle-only", metavar="OUT",
                    help="CPU side only (no GPU): build the oracle, write its sample digests, counters and "
                         "CPU baseline to OUT (JSON). At config 5's full size the oracle and the engine's "
                         "host mirror do not fit one process's memory cap together")
    ap.add_argument("--oracle-file", metavar="IN",
                    help="GPU run: take the parity sample, counters and CPU baseline from a --oracle-only "
                         "file of the same workload instead of building the oracle here")
    args = ap.parse_args()
    heartbeat()
    import faulthandler  # (every thread's stack every 2 minutes: a stall names itself)
    faulthandler.dump_traceback_later(120, repeat=True, file=sys.stderr)
    from mqmatch import workload as W

    t0 = time.time()
    rb, ro, hd, rh = W.gen_retained(args.retained, n_sys=args.sys, seed=W.BASE_SEED + 3)
    fb, fo = W.gen_msg_filters(rh, args.filters, seed=W.BASE_SEED + 4)
    n = len(fo) - 1
    log(f"generated {len(ro) - 1} retained topics, {n} filters in {time.time() - t0:.1f}s")
    if args.oracle_only:
        del rh

        def write(o):
            o = dict(o, retained=len(ro) - 1, filters=n)
            with open(args.oracle_only + ".tmp", "w") as f:
                json.dump(o, f)
            os.replace(args.oracle_only + ".tmp", args.oracle_only)
            log(f"oracle side written to {args.oracle_only} (cpu baseline: {'yes' if o['cpu'] else 'not yet'})")
        write(oracle_side(rb, ro, hd, fb, fo, n, args, early=write))
        return
    import torch
    from mqmatch import engine as E
    torch.cuda.set_device(0)
    t0 = time.time()
    eng = E.Engine(device=0)
    if args.walk:
        eng.set_option(E.OPT_MSG_IMAGE, 0)
    if args.no_img_edges:
        eng.set_option(E.OPT_MSG_EDGES, 0)
    if args.export != 1:
        eng.set_option(E.OPT_MSG_EXPORT, args.export)
    if args.no_key_index:
        eng.set_option(E.OPT_MSG_KEYIDX, 0)
    elif args.key_index_rounds >= 2:
        eng.set_option(E.OPT_MSG_KEYIDX, args.key_index_rounds)
    eng.retain_bulk(rb, ro, hd)
    log(f"engine index built in {time.time() - t0:.1f}s: {eng.stats()}")
    stream = torch.cuda.current_stream()
    d_fb = torch.from_numpy(np.concatenate([fb, np.zeros(16, np.uint8)])).to("cuda:0")
    d_fo = torch.from_numpy(fo.view(np.int64)).to("cuda:0")
    eng.sync(stream.cuda_stream)
    torch.cuda.synchronize()

    runs = args.format == "runs"

    def step():
        if runs:
            return eng.messages_runs_device(d_fb.data_ptr(), d_fo.data_ptr(), n, stream.cuda_stream)
        return eng.messages_device(d_fb.data_ptr(), d_fo.data_ptr(), n, stream.cuda_stream)

    eng.profile(True)  # the first step builds the level-order image: timed apart
    for _ in range(args.warmup):
        r = step()
    torch.cuda.synchronize()
    _pb = eng.profile_read()
    build, kxb = _pb.get("msg_image"), _pb.get("msg_kx_build")
    eng.profile_reset()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        r = step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    prof = eng.profile_read()
    eng.profile(False)
    # one more, untimed step with the count pass's work counters (MQ_PROF_WORK: image edge-table
    # lookups of the fan-outs, for the roofline's bytes)
    eng.profile(True, work=True)
    eng.profile_reset()
    step()
    torch.cuda.synchronize()
    wk = eng.profile_read()
    eng.profile(False)
    lookups = wk.get("msg_fanout_lookups", (0, 0.0))[0]
    r = step()  # (the result the parity checks read: a plain step's)
    torch.cuda.synchronize()
    handles = int(r.n_expanded) if runs else int(r.n_handles)
    out = {
        "metric": "Messages filters/sec (retained reverse match)", "value": n * args.steps / elapsed,
        "unit": "filters/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True, "dtype": "u64",
        "data": "synthetic (SURVEY.md §8d generator, retained seed +3)",
        "config": {"workload": f"config 5 scaled: {len(ro) - 1} retained topics ({args.sys} $SYS), "
                               f"{n} wildcard filters per step", "retained": len(ro) - 1, "filters": n},
        "format": args.format, "handles_per_step": handles, "handles_per_filter": handles / max(1, n),
        "runs_per_step": int(r.n_runs_total) if runs else None,
        "fanout_lookups_per_step": lookups,
        "count_pass_filter_clocks": {k[len("msg_cyc16_"):]: 16 * wk[k][0] for k in wk if k.startswith("msg_cyc16_")},
        "count_pass_lane_walks": {"filters": wk.get("msg_lane_walk_filters", (0, 0))[0],
                                  "particles": wk.get("msg_lane_walk_particles", (0, 0))[0]},
        "kernels_ms_per_step": {k: v[1] / args.steps for k, v in prof.items() if v[1] > 0},
        "path": "particle walk (k_msg)" if args.walk else ("level-order image (k_msgq" + (", runs out" if runs else " + k_msg_copy") + "), literal lookups "
                                                          + ("through the index's edge table" if args.no_img_edges
                                                             else "in the image's edge table")
                                                          + ("" if args.no_key_index else "; under wide runs the key index")),
        "image_build_ms": (build[1] if build else 0.0) + (kxb[1] if kxb else 0.0) if build else None,
        "image_build_parts_ms": {"image": build[1] if build else None, "key_index": kxb[1] if kxb else None},
    }
    cpu = None
    o = None
    if args.oracle_file:
        with open(args.oracle_file) as f:
            o = json.load(f)
        if o["retained"] != len(ro) - 1 or o["filters"] != n:
            raise SystemExit(f"{args.oracle_file} is for another workload")
        out["oracle_side"] = f"{args.oracle_file} (bench_messages.py --oracle-only, same seeds and sizes)"
    elif not args.no_cpu:
        o = oracle_side(rb, ro, hd, fb, fo, n, args)
    if o is not None:
        ns = o["sample_filters"]
        dg = np.array([int(x, 16) for x in o["digests"]], np.uint64)
        cnt = np.array(o["counts"], np.uint32)
        if "all_digests" in o:
            t0 = time.time()
            if runs:  # the timed batch's own device result, every filter
                sys.path.insert(0, os.path.join(REPO, "oracle"))
                import oracle as O
                dres = E.device_messages_runs(r, n)
                want = np.array([int(x, 16) for x in o["all_digests"]], np.uint64)
                wcnt = np.array(o["all_counts"], np.uint64)
                bad_c = int((dres["count"].astype(np.uint64) != wcnt).sum())
                bad_d = int((O.run_digests(dres, nthreads=16) != want).sum())
                out["parity_all"] = {"filters": n, "result": "the last timed step's device runs (mq_messages_runs_device)",
                                     "counts_differ": bad_c, "digests_differ": bad_d,
                                     "digests_equal": bad_c == 0 and bad_d == 0,
                                     "against": o.get("all_note", "fast restatement")}
                del dres
            else:
                out["parity_all"] = full_parity(eng, fb, fo, o)
            log(f"parity over all {n} filters in {time.time() - t0:.1f}s: {out['parity_all']}")
        # (after parity_all, which reads the timed step's device result: this batch overwrites it)
        if runs:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle as O
            res = eng.messages_runs_batch(fb, fo[:ns + 1])
            out["parity_sample"] = {"filters": ns, "counts_equal": bool((res["count"] == cnt).all()),
                                    "digests_equal": bool((O.run_digests(res) == dg).all()),
                                    "result": "mq_messages_runs_batch (host runs)"}
            del res
        else:
            base, count, hs = eng.messages_batch(fb, fo[:ns + 1])
            out["parity_sample"] = {"filters": ns, "counts_equal": bool((count == cnt).all()),
                                    "digests_equal": bool((handle_digests(base, count, hs) == dg).all())}
            del base, count, hs
        per = o["per_filter"]
        b = 8 * per["L"] + 4 + 16 * per["P"] + 16 * per["O"]
        out["alg_bytes_per_filter"] = {"B": b, **per, "sample_filters": ns}
        kms = sum(v[1] for k, v in prof.items() if k.startswith("msg") and k != "msg_image") / args.steps
        if kms > 0:
            # The image path's own algorithmic bytes: the filter's bytes and offset, and every
            # emitted handle read once from the image and written once to the output. SURVEY
            # §8d's B also prices the reference walk's child enumerations (16·P), which the image
            # path does not perform: that rate is reported beside it (it can exceed HBM peak).
            if runs:
                # what the runs path reads and writes: the filter (8 B per level) and a 32 B image
                # edge slot per literal level, a 32 B slot per fan-out lookup (work counter), the
                # image's child range (16 B) and live prefix (16 B) per run, the run written (16 B)
                # and each filter's run base, run count, base and count (24 B + 4 B offset)
                rpf = int(r.n_runs_total) / max(1, n)
                b_img = 40 * per["L"] + 28 + 32 * lookups / max(1, n) + 48 * rpf
                bytes_note = ("40 B per level (filter bytes + an image edge slot), 28 B per filter, 32 B per fan-out "
                              "lookup, 48 B per run (children range, live prefix, the run written)")
            else:
                b_img = 8 * per["L"] + 4 + 16 * int(r.n_handles) / max(1, n)
                bytes_note = "8 B per level + 4 B offset per filter, 16 B per emitted handle (read + write)"
            ach = b_img * n / (kms * 1e-3) / 1e9
            traffic = read_msg_traffic(args.retained, n, args.format, not args.no_key_index, args.export) if not args.walk else None  # (keyed by --retained)
            out["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                               "kernel": ("k_msgq (count, wide count, place, wide place)" + ("" if runs else " + k_msg_copy")
                                          if not args.walk else "k_msg (count + fill)"),
                               "bytes": bytes_note, "bytes_per_step": b_img * n, "ms_per_step": kms}
            if traffic:  # the measured HBM bytes (calibrated PMC, profiles/pmc_traffic.json) over the same time
                out["roofline"]["hbm_traffic_GBps"] = traffic / (kms * 1e-3) / 1e9
                out["roofline"]["hbm_traffic_frac"] = out["roofline"]["hbm_traffic_GBps"] / HBM_PEAK_GBS
            out["survey_B_rate"] = {"GBps": b * n / (kms * 1e-3) / 1e9,
                                    "note": "SURVEY 8d B (incl. 16 B per child enumeration of the reference walk) "
                                            "per step time: the reference's work rate, not HBM traffic"}
        cpu = o["cpu"]
    out["cpu_baseline"] = cpu
    try:
        with open("/proc/self/status") as f:
            hwm = [l.split()[1] for l in f if l.startswith("VmHWM")]
        log(f"peak host memory: {int(hwm[0]) / 2**20:.1f} GiB")
    except (OSError, IndexError, ValueError):
        pass
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
