"""Summarise rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, one counter per run) per kernel: the
per-dispatch mean in KB as rocprofv3 reports it, and in bytes (x1024) — FETCH_SIZE taken x1 for
random-probe kernels and x2 for coalesced streams (calibration: profiles/pmc_traffic.json).

  python tools/pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> > pmc.json
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fd = sum(f) / len(f) if f else 0.0
        wd = sum(w) / len(w) if w else 0.0
        out[k] = {"FETCH_SIZE": {"total": sum(f), "dispatches": len(f), "per_dispatch": fd},
                  "WRITE_SIZE": {"total": sum(w), "dispatches": len(w), "per_dispatch": wd},
                  "hbm_bytes_per_dispatch": {"fetch_raw": fd * 1024, "fetch_corrected_x2": 2 * fd * 1024,
                                             "write": wd * 1024, "total_random_x1": (fd + wd) * 1024,
                                             "total_corrected": (2 * fd + wd) * 1024}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
