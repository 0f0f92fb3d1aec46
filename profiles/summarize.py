"""Summarise rocprofv3 CSV output (kernel trace / stats / PMC counter collection) into the
per-kernel tables kept under profiles/.

  python profiles/summarize.py gpurun_out/prof_1m           # kernel_stats + trace summary
  python profiles/summarize.py gpurun_out/pmc1 gpurun_out/pmc2 --pmc

HBM bytes follow MI355X_MICROARCH.md's HBM/rocprofv3 section: FETCH_SIZE and WRITE_SIZE are
in KiB, come from separate passes. FETCH_SIZE tallies 64 B per L2-to-fabric read request: a wide
coalesced stream issues 128 B requests (x2, "corrected"), random sub-line loads 64 B ones (x1,
"random"; calibrated with tools/randbench on the GPU, profiles/r03/walk_frontier/rb_pmc.json).
"""
import collections
import csv
import glob
import json
import os
import sys


def kernel_stats_db(path):
    """Kernel stats from a rocprofv3 SQLite database (the default output format of ROCm 7)."""
    import sqlite3
    c = sqlite3.connect(path)
    out = []
    for name, calls, total, avg, pct in c.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        out.append({"kernel": name.split("(")[0], "calls": int(calls), "avg_us": float(avg),
                    "total_ms": float(total) / 1e3, "pct": float(pct)})
    return out


def kernel_stats(d):
    out = []
    for path in glob.glob(os.path.join(d, "*.db")):
        out.extend(kernel_stats_db(path))
    for path in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        for r in csv.DictReader(open(path)):
            out.append({"kernel": r["Name"].split("(")[0], "calls": int(r["Calls"]),
                        "avg_us": float(r["AverageNs"]) / 1e3, "total_ms": float(r["TotalDurationNs"]) / 1e6,
                        "pct": float(r["Percentage"])})
    return out


def pmc(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(path)):
                k = r["Kernel_Name"].split("(")[0]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                calls[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    out = {}
    for k, v in agg.items():
        e = {}
        for c, x in v.items():
            n = len(calls[(k, c)])
            e[c] = {"total": x, "dispatches": n, "per_dispatch": x / max(1, n)}
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            nf, nw = len(calls[(k, "FETCH_SIZE")]), len(calls[(k, "WRITE_SIZE")])
            fetch = v["FETCH_SIZE"] * 1024 / max(1, nf)
            write = v["WRITE_SIZE"] * 1024 / max(1, nw)
            # FETCH_SIZE = 64 B per read request: x2 for 128 B streaming requests, x1 for the 64 B
            # requests of random sub-line loads (calibrated with tools/randbench, pmc_traffic.json)
            e["hbm_bytes_per_dispatch"] = {"fetch_raw": fetch, "fetch_corrected_x2": 2 * fetch,
                                           "write": write, "total_corrected": 2 * fetch + write,
                                           "total_random_x1": fetch + write}
        out[k] = e
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--pmc" in sys.argv:
        print(json.dumps(pmc(args), indent=1))
    else:
        for d in args:
            print(json.dumps(kernel_stats(d), indent=1))
