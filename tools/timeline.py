"""Print the kernel timeline of the last match step from a rocprofv3 kernel trace (CSV):
start / end (ms from the first dispatch), duration and queue of every engine kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
mine = [r for r in rows if r["Kernel_Name"].startswith(("mq::", "void mq::", "__amd"))]
walks = [i for i, r in enumerate(mine) if "k_walk" in r["Kernel_Name"]]
last = mine[walks[-1] - 2:] if walks else mine
s0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'].split('(')[0][:34]:34s} queue {r['Queue_Id']:>3s} "
          f"{(s - s0) / 1e6:8.2f} {(e - s0) / 1e6:8.2f} ms  {(e - s) / 1e6:7.2f} ms")
print(f"step span {(int(last[-1]['End_Timestamp']) - s0) / 1e6:.2f} ms")
