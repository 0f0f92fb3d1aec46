"""Print the headline fields of bench JSON lines (development helper)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except (OSError, ValueError) as e:
        print(f, "unreadable:", e)
        continue
    k = {a: round(b, 2) for a, b in d.get("kernels_ms_per_step", {}).items()}
    r = d.get("roofline") or {}
    print(f"{f}: {d['value']/1e6:.2f} M/s  {d['ms_per_step']:.2f} ms/step  {k}  copy {r.get('achieved') or 0:.0f} GB/s")
