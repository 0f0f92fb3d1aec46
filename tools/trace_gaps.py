"""Kernel timeline of a rocprofv3 --kernel-trace CSV: per kernel name the mean duration, and the
mean idle gap before it (its start minus the previous kernel's end on the same queue) over the
last N dispatches of a steady-state run.

  python tools/trace_gaps.py <run_kernel_trace.csv> [last_n]
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-last:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        dur[k].append(e - s)
        if prev_end is not None:
            gap[k].append(s - prev_end)
        prev_end = e
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    busy = sum(sum(v) for v in dur.values())
    print(f"{len(rows)} dispatches over {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / span:.1f} %)")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        d, g = dur[k], gap.get(k, [0])
        print(f"{len(d):5d}  {sum(d) / len(d) / 1e3:8.2f} us  gap before {sum(g) / len(g) / 1e3:7.2f} us  {k}")


if __name__ == "__main__":
    main()
