"""Benchmark: matched publishes/sec of the MI355X TopicsIndex engine (BASELINE.json metric).

A step is one pass of the hot path over one batch: Subscribers() for every topic of a
1M-topic publish batch already resident in HBM. Default (--format spans, mq_match_spans_device):
walk, scan, k_desc (one span per gathered particle list) and k_merge (every record whose row
differs from the stored subscription resolved into a patch: Subscription.Merge across the
client's matches, the '$' rule, inline last-write) — the complete Subscribers result of every
topic, the gathered lists named rather than copied. --format rows materialises
every row (mq_match_device_chunks, each chunk consumed by a device-side checksum). The index
(10M subscriptions, config-2/3 mix) is built through the C-ABI bulk path.

Multi-GPU (`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`): one process
per GPU, the index replicated on every GPU and each rank matching its own 1M-topic batch —
topics are independent units, so there is no data-path collective ("scaling": "weak"); only
the timing barrier and a max-over-ranks all-reduce of the elapsed time use the process group.
`--shard filter` runs the north-star sharded mode instead (subscriptions sharded by filter hash,
every rank matching the full batch, cross-shard lists all-gathered over RCCL each step).

Rank 0 prints one JSON line with the roofline of the dominant kernel (spans: k_merge; rows:
k_copy; HIP events on its launch stream; PMC traffic from profiles/pmc_traffic.json) and the CPU
baseline (the fast CPU restatement of the Go trie on all allotted host cores, on a bounded
sample of the same batch).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mqtt-server_amd"))

METRIC = "matched publishes/sec (whole node) at 10M subs; HBM GB/s fraction of peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

PIPE_BATCHES = 8  # batches per timed run of the pipelined end-to-end leg
WALK_TRIAL_MIN = 65536  # device.h kWalkTrialMin: batches this large run the engine's walk trials
WALK_TRIAL_BATCHES = 6  # device.h kWalkTrialSeq: untimed F, T, then timed T, F, F, T

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
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _device_view(ptr, nbytes):
    """A torch uint8 tensor over library-owned device memory (__cuda_array_interface__)."""
    import torch

    class _Buf:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (int(ptr), False),
                                    "version": 3, "strides": None}
    return torch.as_tensor(_Buf(), device="cuda")


def affinity_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def host_cores():
    """Host threads for the CPU baseline: every core this process may use (the GOMAXPROCS
    analogue), capped by OMP_NUM_THREADS where the machine sets this job's share of a shared
    host (the GPU box shows all of its CPUs to every job but allots 16 per GPU, sets
    OMP_NUM_THREADS=16 and asks that worker pools stay within it)."""
    n = affinity_cpus()
    cap = os.environ.get("OMP_NUM_THREADS", "")
    if cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def read_traffic(path, n_subs, write_bytes_per_launch):
    """HBM bytes per k_copy launch (FETCH_SIZE x2 + WRITE_SIZE) from a committed rocprofv3 PMC
    summary of the same configuration, if present: the entry is used only when its WRITE_SIZE per
    launch is within 5 % of this run's algorithmic bytes per launch (same chunking)."""
    try:
        with open(path) as f:
            e = json.load(f).get(str(n_subs))
        if e is None or abs(float(e["write"]) - write_bytes_per_launch) > 0.05 * write_bytes_per_launch:
            return None
        return float(e["hbm_bytes_per_copy_launch"])
    except (OSError, ValueError, KeyError, TypeError):
        return None


def read_spans_traffic(path, n_subs, n_topics):
    """HBM bytes per step of the k_merge<spans> launches (FETCH_SIZE x2 + WRITE_SIZE, both passes
    with merge-set dedup) from a committed rocprofv3 PMC summary of the same configuration
    (subscriptions, topics per step, dedup), if present."""
    try:
        with open(path) as f:
            e = json.load(f).get("spans_dedup", {}).get(str(n_subs))
        if e is None or int(e["topics"]) != n_topics:
            return None
        return float(e["hbm_bytes_per_step"])
    except (OSError, ValueError, KeyError, TypeError):
        return None


def engine_option(opt, default):
    """An engine option as MQ_ENGINE_OPTIONS sets it for this process (mqmatch/engine.py)."""
    for kv in os.environ.get("MQ_ENGINE_OPTIONS", "").split(","):
        if kv.strip() and int(kv.split("=")[0]) == opt:
            return int(kv.split("=")[1])
    return default


def read_walk_traffic(path, n_subs, n_topics, edge_load, walk_group, fused):
    """HBM bytes per walk launch (FETCH_SIZE x1 + WRITE_SIZE) from a committed rocprofv3 PMC
    summary of the configuration that ran (subscriptions, topics, the index's edge-table load as
    mq_index_stats reports it, the walk the engine's trials chose, the fused desc), if present."""
    try:
        with open(path) as f:
            e = json.load(f).get("walk", {}).get(str(n_subs))
        if (e is None or int(e["topics"]) != n_topics or int(e.get("edge_load", 2)) != int(edge_load)
                or int(e.get("walk_group", 0)) != int(walk_group)
                or int(e.get("fused_desc", 0)) != int(fused)):
            return None
        return float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError, TypeError):
        return None


def walk_roofline(prof, steps, n, n_subs, per_topic, gathers_per_step, edge_load=16, walk_group=16, no_desc=True):
    """Roofline of the match walk, k_walkf (16 lanes per topic), with k_desc fused into its
    epilogue (the default for device results, MQ_OPT_FUSE_DESC). Its algorithmic bytes per topic
    are SURVEY.md §8(d)'s walk terms, 8·L + 4 + 16·P (L levels, P child lookups of the
    reference's DFS, counted exactly by the oracle on a sample of the batch), plus the desc's:
    per gathered particle its 32 B list record and 16 B pair-block header read and its 16 B span
    written, per topic 32 B of counts and signature (the merge lists' 16 B per merge gather are not
    counted: an understatement). Unfused (MQ_OPT_FUSE_DESC 0): the walk terms plus the 4 B gather
    word per gathered particle. Over its mean launch time from HIP events in the timed region.
    Dependent probes of a 4 GB edge table: bound by random-access latency and request rate, far
    below streaming bandwidth."""
    launches, ms = prof.get("walk", (0, 0.0))
    fused = engine_option(17, 1) != 0 and no_desc
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
            "traffic": None,
            "kernel": "k_walkf (frontier walk, 16 lanes per topic) + k_desc fused" if fused
                      else "the match walk (k_walkf frontier or k_walk thread per topic, whichever the engine's "
                           "trial batches found faster), count pass",
            "bytes": ("8 B per level + 4 B offset + 16 B per child lookup (SURVEY 8d: 8L + 4 + 16P) + 64 B per "
                      "gathered particle (list record, pair header, span) + 32 B per topic") if fused else
                     "8 B per level + 4 B offset + 16 B per child lookup (SURVEY 8d: 8L + 4 + 16P) + 4 B per gather word"}
    if not launches or ms <= 0 or per_topic is None:
        return roof
    b_topic = 8 * per_topic["L"] + 4 + 16 * per_topic["P"]
    per_launch = (b_topic + 32) * n + 64 * gathers_per_step if fused else b_topic * n + 4 * gathers_per_step
    launch_ms = ms / launches
    achieved = per_launch / (launch_ms * 1e-3) / 1e9
    traffic = read_walk_traffic(os.path.join(REPO, "profiles", "pmc_traffic.json"), n_subs, n, edge_load,
                                walk_group, 1 if fused else 0)
    roof["traffic_key"] = {"subs": n_subs, "topics": n, "edge_load": edge_load, "walk_group": walk_group,
                           "fused_desc": 1 if fused else 0}
    roof.update(achieved=achieved, frac=achieved / HBM_PEAK_GBS, launch_ms=launch_ms, bytes_per_launch=per_launch,
                traffic=traffic)
    if traffic:  # the measured HBM bytes (calibrated PMC) over the same launch time
        roof["hbm_traffic_GBps"] = traffic / (launch_ms * 1e-3) / 1e9
        roof["hbm_traffic_frac"] = roof["hbm_traffic_GBps"] / HBM_PEAK_GBS
    return roof


def spans_roofline(prof, work, steps, n, n_subs):
    """Roofline of the span format's merge stage, k_merge<spans>: with merge-set dedup (the
    default) two launches per step — the set pass (one resolution per distinct merge set) and the
    topic pass (the topics k_finish left: inline rows, or beyond the dedup). Its algorithmic bytes
    per step are what the two launches read and write for the topics they resolve
    (k_finish, a separate kernel, writes every other topic's record): 64 B per topic resolved
    (its counts and set slot read, its result record or SetInfo written), its map's sources (16 B
    per merge gather from the dedup lists, or the 32 B GDesc of every gather), 16 B per
    pair-table entry probed, 16 B per pair slot resolved, 8 B per partner link, 8 B per patch —
    priced from the work counters of an extra step (the same batch, so the same work) — over the
    two launches' time from HIP events in the timed region. Latency-bound (dependent probes of hash tables and
    lists), so the HBM fraction is low by nature; the step's other kernels are walk, desc, dedup."""
    launches, ms = prof.get("merge", (0, 0.0))
    set_launches, set_ms = prof.get("merge_sets", (0, 0.0))
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
            "traffic": None, "kernel": "k_merge<spans>" + (" (set pass + topic pass)" if set_launches else ""),
            "bytes": "per topic resolved: counts + result/SetInfo + map sources; pair entries + pair slots + "
                     "partner links + patches"}
    if not launches or ms <= 0:
        return roof
    g = lambda k: work.get(k, (0, 0.0))[0]
    per_step = (64 * g("merge_topics_resolved") + g("merge_map_bytes") + 16 * g("merge_pair_entries")
                + 16 * g("merge_records") + 8 * g("merge_links") + 8 * g("merge_patches"))
    step_ms = (ms + set_ms) / max(1, steps)
    achieved = per_step / (step_ms * 1e-3) / 1e9
    traffic = read_spans_traffic(os.path.join(REPO, "profiles", "pmc_traffic.json"), n_subs, n) if set_launches else None
    # the work counters themselves, and the set pass's phase clocks (shader clocks summed over its
    # wavefronts: map, pair analysis, resolution of the records, whole set)
    roof["work"] = {k: g(k) for k in ("merge_pair_entries", "merge_records", "merge_links", "merge_patches",
                                      "merge_topics_resolved", "set_cycles_map", "set_cycles_pairs",
                                      "set_cycles_resolve", "set_cycles_total")}
    roof.update(achieved=achieved, frac=achieved / HBM_PEAK_GBS, ms_per_step=step_ms,
                launches_per_step=(launches + set_launches) / max(1, steps),
                launch_ms_avg=(ms + set_ms) / max(1, launches + set_launches), bytes_per_step=per_step,
                traffic=traffic)
    if traffic:  # most algorithmic bytes are cache hits: the measured HBM bytes over the same time
        roof["hbm_traffic_GBps"] = traffic / (step_ms * 1e-3) / 1e9
        roof["hbm_traffic_frac"] = roof["hbm_traffic_GBps"] / HBM_PEAK_GBS
    return roof


def rows_roofline(prof, args, elapsed, out):
    """Roofline of the row format's dominant kernel, k_copy. It moves every gathered list into
    output rows: per launch it writes copy_bytes (16 B per client row, 8 B per shared / inline
    row), all of which must reach HBM (the rows of one step are far larger than every cache).
    Its reads are the hot subscription lists, re-read by many topics and served from L2 / the
    Infinity Cache, so the HBM-compulsory bytes of a launch are its writes;
    `traffic` is the PMC-measured HBM bytes per launch (profiles/pmc_traffic.json) when present."""
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
            "traffic": None, "kernel": "k_copy", "bytes": "output rows written per launch"}
    copy_launches, copy_ms = prof.get("copy", (0, 0.0))
    copy_bytes = prof.get("copy_bytes", (0, 0.0))[0]
    if copy_ms > 0 and copy_launches:
        launch_ms = copy_ms / copy_launches
        per_launch = copy_bytes / copy_launches
        achieved = per_launch / (launch_ms * 1e-3) / 1e9
        roof.update(achieved=achieved, frac=achieved / HBM_PEAK_GBS,
                    traffic=read_traffic(os.path.join(REPO, "profiles", "pmc_traffic.json"), args.subs, per_launch))
        out["copy_avg_launch_ms"] = launch_ms
        out["copy_bytes_per_launch"] = per_launch
        # the whole step against the same roofline: all output bytes / step time
        out["step_output_GBps"] = copy_bytes / max(1, args.steps) / (elapsed / args.steps) / 1e9
    return roof


def run_sharded(args, mix, n_clients, rank, world, local, backend):
    """North-star sharded mode. A step is one batch of
    --topics publish topics matched by the whole node: every shard walks the full batch
    (mq_match_spans_begin), the shards all-gather their exported cross-shard node lists (RCCL
    all-gather over xGMI via torch.distributed; --sim-shards: through device memory on one GPU),
    and each shard resolves its own subscriptions exactly (mq_match_spans_end). The topic's
    Subscribers are the union of the shards' disjoint results. Total work per step is fixed as
    shards are added ("scaling": "strong")."""
    import numpy as np
    import torch
    from mqmatch import dist as D
    from mqmatch import engine as E
    from mqmatch import workload as W
    sim = args.sim_shards if world == 1 else 0
    n_shards = sim or world
    t0 = time.time()
    w = W.gen_subscriptions(args.subs, n_clients, seed=W.BASE_SEED, mix=mix)
    log(f"generated {args.subs} subscriptions in {time.time()-t0:.1f}s")
    t0 = time.time()
    mine = range(n_shards) if sim else [rank]
    engs = [E.Engine(device=local, expected_subs=args.subs // n_shards, shard=k, n_shards=n_shards) for k in mine]
    for e in engs:
        e.subscribe_bulk(w)
    log(f"{len(engs)} shard index(es) built in {time.time()-t0:.1f}s: {[e.stats() for e in engs]}")
    tb, to = W.gen_topics(w, args.topics, seed=D.topic_seed(0), mix=mix)  # the same batch on every shard
    n = len(to) - 1
    stream = torch.cuda.current_stream()
    d_tb = torch.from_numpy(tb).to(f"cuda:{local}")
    d_to = torch.from_numpy(to.view(np.int64)).to(f"cuda:{local}")
    for e in engs:
        e.sync(stream.cuda_stream)
    torch.cuda.synchronize()
    ents = []

    def step():
        xs = [e.match_spans_begin(d_tb.data_ptr(), d_to.data_ptr(), n, stream.cuda_stream) for e in engs]
        ents.append(sum(int(x.n_ents) for x in xs))
        if sim:
            for k, e in enumerate(engs):
                e.match_spans_end([x for j, x in enumerate(xs) if j != k], stream.cuda_stream)
        else:
            foreign, keep = D.exchange_xlists(xs[0], backend) if backend else ([], None)
            engs[0].match_spans_end(foreign, stream.cuda_stream)
            del keep

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # the timed steps carry no HIP events (each record is on a step's critical path: a shard's
    # begin and end synchronise once each); the kernels' times come from an untimed pass after
    ents.clear()
    D.barrier(backend)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    D.barrier(backend)
    elapsed = D.max_over_ranks(time.perf_counter() - t_start, backend)
    ents_step = D.sum_over_ranks(sum(ents) / max(1, args.steps), backend)
    kb = min(args.steps, 20)
    for e in engs:
        e.profile(True)
        e.profile_reset()
    for _ in range(kb):
        step()
    torch.cuda.synchronize()
    profs = [e.profile_read() for e in engs]
    for e in engs:
        e.profile(False)
    if rank != 0:
        D.finalize(backend)
        return
    kern = {}
    for p in profs:
        for k, v in p.items():
            if v[1] > 0:
                kern[k] = kern.get(k, 0.0) + v[1] / max(1, kb) / len(profs)
    ms = 1000.0 * elapsed / args.steps
    out = {
        "metric": METRIC, "value": n / (elapsed / args.steps), "unit": "publishes/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (SURVEY.md §8d generator, seed 0x6D716D61)",
        "config": {"workload": f"config-3 mix: {args.subs} subscriptions sharded by filter hash over {n_shards} shards, "
                               f"{n} publish topics per step matched by every shard",
                   "subs": args.subs, "clients": n_clients, "topics_per_step": n, "shards": n_shards,
                   "parallelism": (f"{n_shards} shards simulated on one GPU (run in turn; exchange through device "
                                   f"memory)" if sim else f"one shard per GPU, RCCL all-gather of the cross-shard lists"),
                   "format": "spans"},
        "kernels_ms_per_step_per_shard": kern,
        "kernels_pass": f"HIP events around every kernel in an untimed pass of {kb} steps; the timed steps carry none",
        "exchange": {"entries_per_topic": ents_step / n,
                     "bytes_per_topic_exported": 16.0 * ents_step / n + 4.0 * n_shards,
                     "note": "each shard exports 4 B of count + 16 B per cross-shard node per topic; an all-gather "
                             "delivers every other shard's export to each shard"},
        "roofline": None, "cpu_baseline": None,
    }
    if sim:
        out["note"] = ("simulated shards run one after another on one GPU: ms_per_step is the sum of the shards' "
                       "work, so a node with one shard per GPU would run a step in about ms_per_step / shards "
                       "plus the exchange")
    print(json.dumps(out), flush=True)
    D.finalize(backend)


class OracleSide:
    """The CPU side of the bench line — the oracle's parity-sample digests and L / P / S / O
    counters, and the CPU baselines — in a child process (`bench.py --oracle-side`) started
    before this process touches the GPU. It regenerates the same workload from the same seeds,
    builds the oracle while the engine is built and timed here, and times the CPU baselines only
    when told to (finish()), so that they do not share the host with this process's work. At
    config 4's 50M subscriptions the oracle and the engine's host mirror live in two processes."""

    def __init__(self, args):
        import subprocess
        import tempfile
        self.path = os.path.join(tempfile.gettempdir(), f"mq_oracle_side_{os.getpid()}.json")
        cmd = [sys.executable, "-u", os.path.abspath(__file__), "--oracle-side", self.path,
               "--subs", str(args.subs), "--clients", str(args.clients), "--mix", args.mix,
               "--topics", str(args.topics), "--cpu-seconds", str(args.cpu_seconds),
               "--parity-topics", str(args.parity_topics)]
        self.p = subprocess.Popen(cmd, stdin=subprocess.PIPE)

    def finish(self, timeout=1800):
        self.p.stdin.write(b"go\n")
        self.p.stdin.flush()
        self.p.stdin.close()
        rc = self.p.wait(timeout=timeout)
        if rc != 0:
            raise SystemExit(f"bench.py --oracle-side failed (rc {rc})")
        with open(self.path) as f:
            o = json.load(f)
        os.unlink(self.path)
        return o


def oracle_side_main(args):
    """Child process of OracleSide: no torch, no GPU."""
    from mqmatch import dist as D
    from mqmatch import workload as W
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    mix = W.MIX_IOT if args.mix == "iot" else W.MIX_MQTT
    n_clients = args.clients or (args.subs if args.mix == "iot" else max(1, args.subs // 10))
    t0 = time.time()
    w = W.gen_subscriptions(args.subs, n_clients, seed=W.BASE_SEED, mix=mix)
    tb, to = W.gen_topics(w, args.topics, seed=D.topic_seed(0), mix=mix)
    n = len(to) - 1
    log(f"oracle side: workload generated in {time.time()-t0:.1f}s")
    t0 = time.time()
    orc = O.OracleIndex()
    orc.subscribe_bulk(w)
    del w
    log(f"oracle side: oracle index built in {time.time()-t0:.1f}s")
    cores = host_cores()
    # oracle counters (B = 8L + 4 + 16P + 16S + 16O per topic) + parity digests
    ns = min(n, args.parity_topics)
    t0 = time.time()
    dg_o, cnt_o, tot = orc.digest_batch(tb, to[:ns + 1], cores)
    log(f"oracle side: {ns} sample digests in {time.time()-t0:.1f}s; waiting for the GPU side")
    if sys.stdin.readline().strip() != "go":  # the GPU side is done: the host is this process's
        log("oracle side: the GPU side went away; exiting")
        return
    # The baseline is the fast restatement (oracle/topics_fast.h: the Go trie's algorithm with
    # client ids interned at build time and flat per-thread result tables; digest-equal to the
    # oracle): calibrate, then time a sample of about --cpu-seconds of CPU work.
    t0 = time.time()
    fast = orc.fast()
    log(f"oracle side: fast CPU restatement built in {time.time()-t0:.1f}s")
    cal = min(n, 256 * cores)
    secs, _ = fast.bench_subscribers(tb, to[:cal + 1], cores)
    m = int(min(n, max(cal, cal * args.cpu_seconds / max(secs, 1e-6))))
    secs, _ = fast.bench_subscribers(tb, to[:m + 1], cores)
    # one thread on a short sample: the per-core rate (the restatement scales with threads: a
    # shared frozen index, no locks), for reading the baseline against a whole host
    m1 = int(min(n, max(64, (m / max(cores, 1)) * min(3.0, args.cpu_seconds / 5) / max(args.cpu_seconds, 1e-6))))
    secs1, _ = fast.bench_subscribers(tb, to[:m1 + 1], 1)
    cpu = {"value": m / secs, "unit": "publishes/s", "cores": cores, "kind": "port",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "affinity_cpus": affinity_cpus(),
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
           "single_thread": {"value": m1 / secs1, "sample_topics": m1},
           "sample": f"first {m} topics of the rank-0 batch on the same {args.subs}-subscription index, "
                     f"{cores} threads (std::thread, shared frozen index), Subscribers() per topic: the "
                     f"fast CPU restatement of the Go particle trie (oracle/topics_fast.cpp: interned "
                     f"client ids, flat per-thread result tables; digest-equal to the oracle)"}
    del fast
    # the literal restatement (per-call ordered result maps, as the oracle checks with)
    lit_cal = min(n, 16 * cores)
    lsecs, _ = orc.bench_subscribers(tb, to[:lit_cal + 1], cores)
    lm = int(min(n, max(lit_cal, lit_cal * min(5.0, args.cpu_seconds / 3) / max(lsecs, 1e-6))))
    lsecs, _ = orc.bench_subscribers(tb, to[:lm + 1], cores)
    lit = {"value": lm / lsecs, "unit": "publishes/s", "cores": cores,
           "sample": f"first {lm} topics; oracle/topics_oracle.cpp (ordered std::map results, string keys, "
                     f"map copy per gather)"}
    with open(args.oracle_side, "w") as f:
        json.dump({"sample_topics": ns, "digests": [format(int(x), "x") for x in dg_o],
                   "counts": cnt_o.astype(np.int64).tolist(), "totals": tot, "cpu": cpu, "cpu_literal": lit}, f)
    log("oracle side: done")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--subs", type=int, default=10_000_000)
    ap.add_argument("--clients", type=int, default=0, help="default: subs/10 (mqtt mix), subs (iot mix)")
    ap.add_argument("--mix", choices=["mqtt", "iot"], default="mqtt",
                    help="mqtt: config-2/3 mix (the metric's); iot: config-4 IoT fan-in (exact device filters + 1%% dashboards)")
    ap.add_argument("--topics", type=int, default=1_000_000, help="publish topics per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--select-shared", action="store_true",
                    help="MQ_CFG_SELECT_SHARED: SelectShared on the device (k_pick) in every step")
    ap.add_argument("--shard", choices=["none", "filter"], default="none",
                    help="filter: the north-star sharded mode (SURVEY.md §8e(ii)) — subscriptions sharded by "
                         "filter hash over the ranks, every rank matching the same full batch, the ranks' "
                         "cross-shard node lists all-gathered over RCCL each step (DESIGN.md §6)")
    ap.add_argument("--sim-shards", type=int, default=0,
                    help="one GPU: hold this many shards in one process and run the sharded step on them in "
                         "turn (exchange through device memory): per-shard work and exchange volume")
    ap.add_argument("--format", choices=["spans", "rows"], default="spans",
                    help="spans: mq_match_spans_device (gathered lists named, merges patched); rows: "
                         "mq_match_device_chunks with every row materialised and each chunk consumed "
                         "by a device-side checksum")
    ap.add_argument("--parity-topics", type=int, default=0,
                    help="topics of the timed batch checked against the oracle (default: 4096; iot mix 20000)")
    ap.add_argument("--oracle-side", metavar="OUT", help=argparse.SUPPRESS)  # OracleSide's child process
    args = ap.parse_args()
    if not args.parity_topics:
        args.parity_topics = 20000 if args.mix == "iot" else 4096
    heartbeat()
    if args.oracle_side:
        return oracle_side_main(args)
    rank, world, _ = (int(os.environ.get(k, d)) for k, d in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")))
    oside = None
    if not args.no_cpu and world == 1 and args.shard == "none" and args.sim_shards <= 1:
        oside = OracleSide(args)  # before any GPU call: the child forks no GPU state

    import torch
    from mqmatch import dist as D
    from mqmatch import engine as E
    from mqmatch import workload as W

    rank, world, local_rank = D.env_rank()
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    local = D.device_for(local_rank)
    torch.cuda.set_device(local)
    backend = D.init(local_rank)
    mix = W.MIX_IOT if args.mix == "iot" else W.MIX_MQTT
    n_clients = args.clients or (args.subs if args.mix == "iot" else max(1, args.subs // 10))
    if args.shard == "filter" or args.sim_shards > 1:
        return run_sharded(args, mix, n_clients, rank, world, local, backend)

    t0 = time.time()
    w = W.gen_subscriptions(args.subs, n_clients, seed=W.BASE_SEED, mix=mix)
    log(f"generated {args.subs} subscriptions ({w['n_unique_filters']} distinct filters) in {time.time()-t0:.1f}s")
    t0 = time.time()
    eng = E.Engine(device=local, expected_subs=args.subs, select_shared=args.select_shared)
    eng.subscribe_bulk(w)
    log(f"engine index built in {time.time()-t0:.1f}s: {eng.stats()}")
    tb, to = W.gen_topics(w, args.topics, seed=D.topic_seed(rank), mix=mix)
    n = len(to) - 1

    stream = torch.cuda.current_stream()
    d_tb = torch.from_numpy(tb).to(f"cuda:{local}")
    d_to = torch.from_numpy(to.view(np.int64)).to(f"cuda:{local}")
    t0 = time.time()
    eng.sync(stream.cuda_stream)
    torch.cuda.synchronize()
    log(f"device image uploaded in {time.time()-t0:.1f}s")

    consumed = []

    def consume(chunk, first, cstream):
        # rows format: every chunk is read on its stream before its buffers are reused (a
        # device-side checksum standing in for a fan-out), so the step delivers every row
        nb = int(chunk.n_sub_rows) * 16
        if nb:
            t = torch.cuda.ExternalStream(cstream)
            with torch.cuda.stream(t):
                v = _device_view(chunk.sub_rows, nb)
                consumed.append(v.view(torch.int64).sum())

    if args.format == "spans":
        def step():
            return eng.match_spans_device(d_tb.data_ptr(), d_to.data_ptr(), n, stream.cuda_stream)
    else:
        def step():
            consumed.clear()
            eng.match_device_chunks(d_tb.data_ptr(), d_to.data_ptr(), n, stream.cuda_stream, consume)

    # The engine's walk trials (device.cpp: one untimed batch per walk, then two timed batches
    # per walk in ABBA order; the faster is kept for this index) run before the warm-up steps, so
    # that no trial batch falls in the timed region whatever --warmup is
    eng.profile(True)
    eng.profile_reset()
    calibration = 0
    trial_prof = {}
    if args.format == "spans" and n >= WALK_TRIAL_MIN:
        for _ in range(2 * WALK_TRIAL_BATCHES):  # (a batch whose one-sync buffers overflowed repeats its trial)
            step()
            calibration += 1
            torch.cuda.synchronize()
            for k, v in eng.profile_read().items():
                if k.startswith("trial_"):  # (summed over the batches: the profile is reset after each)
                    trial_prof[k] = (trial_prof.get(k, (0, 0.0))[0] + v[0], 0.0)
            if any(k.startswith("trial_chose_") for k in trial_prof):
                break
            eng.profile_reset()
    torch.cuda.synchronize()
    eng.profile(False)
    walk_trials = {k: v[0] for k, v in trial_prof.items() if k.startswith("trial_")}
    for k in ("trial_frontier_ps_per_topic", "trial_thread_ps_per_topic"):
        if k in walk_trials:  # (two timed batches each: the mean)
            walk_trials[k] = walk_trials[k] / max(1, walk_trials.get(k.replace("ps_per_topic", "batches"), 1))
    walk_group = engine_option(15, 0 if "trial_chose_thread" in walk_trials else 16)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # the timed steps carry HIP events around the walk's launches only (the roofline's kernel):
    # with one host synchronisation per batch every event record is on the step's critical path
    # (16 of them at 16k topics cost ~10 % of a step); the other kernels' times come from a
    # separate profiled pass below
    eng.profile(True, walk_only=args.format == "spans")
    eng.profile_reset()
    D.barrier(backend)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    D.barrier(backend)
    elapsed = time.perf_counter() - t_start
    prof = eng.profile_read()
    eng.profile(False)
    prof_all, kb = prof, args.steps
    if args.format == "spans":  # every kernel's time: an untimed pass of the same batch
        kb = min(args.steps, 20)
        eng.profile(True)
        eng.profile_reset()
        for _ in range(kb):
            step()
        torch.cuda.synchronize()
        prof_all = eng.profile_read()
        eng.profile(False)
    elapsed = D.max_over_ranks(elapsed, backend)
    chunks = eng.match_chunks()
    log(f"timed {args.steps} steps in {elapsed:.3f}s; kernels {prof}; chunks/step {chunks}")
    try:
        with open("/proc/self/status") as f:
            hwm = [l.split()[1] for l in f if l.startswith("VmHWM")]
        log(f"peak host memory of this rank: {int(hwm[0]) / 2**20:.1f} GiB")
    except (OSError, IndexError, ValueError):
        pass

    if rank != 0:
        D.finalize(backend)
        return

    value = n * world * args.steps / elapsed
    out = {
        "metric": METRIC, "value": value, "unit": "publishes/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (SURVEY.md §8d generator, seed 0x6D716D61)",
        "config": {
            "workload": (f"config-3 mix: {args.subs} subscriptions (depth 4-8, 30% '+', 10% '#', "
                         f"5% $share, 0.1% top-level wildcards), {n} publish topics per GPU per step")
                        if args.mix == "mqtt" else
                        (f"config-4 IoT fan-in: {args.subs} subscriptions (exact dev/r/s/d/telemetry filters, "
                         f"one client each, 1% dashboards dev/r/+/+/telemetry | dev/r/s/#), {n} device topics "
                         f"per GPU per step"),
            "subs": args.subs, "clients": n_clients, "topics_per_gpu": n,
            "parallelism": f"index replicated on {world} GPU(s), topic batch per GPU",
            "select_shared": bool(args.select_shared),
            "format": args.format,
        },
        "kernels_ms_per_step": {k: v[1] / max(1, kb) for k, v in prof_all.items() if v[1] > 0},
        "kernels_pass": ("HIP events around every kernel in an untimed pass of %d steps; the timed steps time "
                         "the walk only" % kb) if prof_all is not prof else "the timed steps",
        "counters_per_step": {k: v[0] / max(1, args.steps) for k, v in prof.items() if v[1] == 0},
        "chunks_per_step": chunks,
        "walk_trials": {"calibration_batches": calibration, "chosen_walk_group": walk_group, **walk_trials},
        "edge_load": int(eng.stats()["edge_load"]),
    }

    if args.format == "spans":
        # One extra, untimed step with k_merge's work counters (MQ_PROF_WORK costs atomics).
        eng.profile(True, work=True)
        eng.profile_reset()
        r_last = step()
        torch.cuda.synchronize()
        work = eng.profile_read()
        eng.profile(False)
        out["roofline"] = spans_roofline(prof_all, work, kb, n, args.subs)
        out["merge_work_per_topic"] = {k[6:]: work[k][0] / n for k in work
                                       if k.startswith("merge_") and k not in ("merge_topics", "merge_sets")}
        if "set_cycles_max" in work:  # the longest merge set's wave (shader clocks) and its records
            out["set_longest"] = {"cycles": work["set_cycles_max"][0], "records": work["set_records_max_wave"][0],
                                  **{k[4:]: work[k][0] for k in ("set_pairs_cycles_max", "set_resolve_cycles_max",
                                                                 "set_gathers_max", "set_hit_lists_max") if k in work},
                                  "cycles_mean": work.get("set_cycles_total", (0, 0))[0]
                                  / max(1, work.get("dedup_sets", (1, 0))[0])}
    else:
        out["roofline"] = rows_roofline(prof, args, elapsed, out)
    cpu = None
    if oside is not None:
        # the oracle side (a child process started before any GPU call): its parity-sample
        # digests and L / P / S / O counters are ready or nearly; the CPU baseline is timed now,
        # with this process idle
        o = oside.finish()
        cpu = o["cpu"]
        out["cpu_baseline_literal"] = o["cpu_literal"]
        ns = o["sample_topics"]
        dg_o = np.array([int(x, 16) for x in o["digests"]], np.uint64)
        tot = o["totals"]
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from digest import engine_digests
        if not args.select_shared:  # picked shared rows are checked by tests/test_gpu_select.py
            # span format: the first ns topics of the measured step's own device result (the whole
            # batch's merge sets), expanded as a device consumer would
            res = (E.expand_device_spans(r_last, n, ns) if args.format == "spans"
                   else eng.match_batch(tb, to[:ns + 1]))
            dg_e, cnt_e = engine_digests(res)
            out["parity_sample"] = {"topics": ns, "format": args.format, "bit_exact": bool((dg_e == dg_o).all()),
                                    "counts_equal": bool((cnt_e.astype(np.int64) == np.array(o["counts"], np.int64)).all()),
                                    "checked": "device result of the timed batch" if args.format == "spans"
                                               else "mq_match_batch",
                                    "oracle": "oracle/topics_oracle.cpp in a child process (bench.py --oracle-side)"}
            if args.format == "spans":
                out["parity_sample"]["set_patch_topics"] = res["set_topics"]
        per_topic = {k: v / ns for k, v in tot.items()}
        b_topic = 8 * per_topic["L"] + 4 + 16 * per_topic["P"] + 16 * per_topic["S"] + 16 * per_topic["O"]
        out["alg_bytes_per_topic"] = {"B": b_topic, "L": per_topic["L"], "P": per_topic["P"],
                                      "S": per_topic["S"], "O": per_topic["O"], "sample_topics": ns}
        if args.format == "spans":
            # `roofline` names the step's dominant kernel: the walk or the merge stage, whichever
            # takes longer per step; the other is reported beside it
            wr = walk_roofline(prof, args.steps, n, args.subs, per_topic,
                               out["counters_per_step"].get("gathers", 0), out["edge_load"], walk_group,
                               "desc" not in prof_all)
            mr = out["roofline"]
            walk_ms = wr.get("launch_ms") or 0.0
            merge_ms = mr.get("ms_per_step") or 0.0
            if walk_ms > merge_ms and wr["achieved"] is not None:
                out["roofline"], out["roofline_merge"] = wr, mr
            else:
                out["roofline_walk"] = wr
        # End-to-end through the host-buffer boundary (H2D of the topics, the kernels, D2H of the
        # results into host memory), reported beside `value`, never as it. Span
        # format: mq_match_spans, and separately with every row of a bounded sample expanded on
        # the host (mq_spans_expand, one thread and all host threads); row format: mq_match_batch
        # on a bounded sample (PCIe-bound).
        if args.format == "spans":
            # the spans through host memory on the step's whole batch (as the headline); the row
            # expansions on its first 200k topics
            eng.match_spans_host(tb, to)
            calls = []
            n_calls = 3 if n >= 262144 else 21  # the median of three calls (21 for small batches) after one untimed
            for _ in range(n_calls):
                t0 = time.perf_counter()
                nbytes, _ = eng.match_spans_host(tb, to)
                calls.append(time.perf_counter() - t0)
            dt = sorted(calls)[len(calls) // 2]
            parts = dict(eng.last_host_bytes)
            # pipelined: consecutive batches, each result's copy beside the next batch's kernels
            # (mq_match_spans_submit / _wait); the median of three runs of PIPE_BATCHES batches after
            # one untimed. Each run pays the pipeline's fill (the first batch's kernels) and drain
            # (the last batch's copy) once: in between a batch costs its copy, ~55 GB/s to host.
            eng.match_spans_pipelined(tb, to, 2)
            pcalls, plogs = [], []
            for _ in range(3):
                t0 = time.perf_counter()
                plog = []
                pbytes = eng.match_spans_pipelined(tb, to, PIPE_BATCHES, log=plog)
                pcalls.append(time.perf_counter() - t0)
                plogs.append(plog)
            pdt = sorted(pcalls)[1]
            ne_h = n
            ne = min(n, 200000)
            t0 = time.perf_counter()
            _, nrows = eng.match_spans_host(tb, to[:ne + 1], expand=True)
            dtx = time.perf_counter() - t0
            th = host_cores()
            t0 = time.perf_counter()
            _, nrows_n = eng.match_spans_host(tb, to[:ne + 1], expand=True, threads=th, block=256)
            dtn = time.perf_counter() - t0
            out["end_to_end"] = {"value": ne_h / dt, "unit": "publishes/s", "sample_topics": ne_h,
                                 "calls_ms": [round(1e3 * c, 3) for c in calls], "per_call": "median",
                                 "pipelined": {"value": PIPE_BATCHES * ne_h / pdt, "unit": "publishes/s", "batches": PIPE_BATCHES,
                                               "topics_per_batch": ne_h, "runs_ms": [round(1e3 * c, 3) for c in pcalls],
                                               "median_run_submit_wait_ms": plogs[sorted(range(3), key=lambda i: pcalls[i])[1]],
                                               "bytes_per_topic": pbytes / ne_h,
                                               "GBps_to_host": PIPE_BATCHES * pbytes / pdt / 1e9},
                                 "result_bytes": nbytes, "bytes_per_topic": nbytes / ne_h, "GBps_to_host": nbytes / dt / 1e9,
                                 "bytes_per_topic_by_array": {k: v / ne_h for k, v in parts.items()},
                                 "expanded": {"value": ne / dtx, "rows": nrows, "host_threads": 1, "sample_topics": ne,
                                              "rows_GBps": 16 * nrows / dtx / 1e9},
                                 "expanded_threads": {"value": ne / dtn, "rows": nrows_n, "host_threads": th, "sample_topics": ne,
                                                      "rows_GBps": 16 * nrows_n / dtn / 1e9}}
        else:
            ne = min(n, 20000)
            eng.match_batch_rows(tb, to[:ne + 1])
            t0 = time.perf_counter()
            rows = eng.match_batch_rows(tb, to[:ne + 1])
            dt = time.perf_counter() - t0
            out["end_to_end"] = {"value": ne / dt, "unit": "publishes/s", "sample_topics": ne,
                                 "result_bytes": 16 * rows[0] + 8 * rows[1] + 8 * rows[2],
                                 "GBps_to_host": (16 * rows[0] + 8 * rows[1] + 8 * rows[2]) / dt / 1e9}
    elif args.format == "spans":
        # without the oracle's L / P counters (--no-cpu, multi-rank) the walk's bytes are not
        # known; the walk is still named when it is the longer kernel (achieved: null)
        wr = walk_roofline(prof, args.steps, n, args.subs, None, out["counters_per_step"].get("gathers", 0),
                           out["edge_load"], walk_group, "desc" not in prof_all)
        walk_ms = prof.get("walk", (0, 0.0))[1] / max(1, args.steps)
        if walk_ms > (out["roofline"].get("ms_per_step") or 0.0):
            wr["launch_ms"] = walk_ms
            wr["note"] = "algorithmic bytes need the oracle's per-topic L / P counters (run without --no-cpu)"
            out["roofline"], out["roofline_merge"] = wr, out["roofline"]
    out["cpu_baseline"] = cpu
    print(json.dumps(out), flush=True)
    D.finalize(backend)


if __name__ == "__main__":
    main()
