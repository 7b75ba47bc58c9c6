"""Summarise a rocprofv3 kernel trace: per-kernel mean duration and the idle
gap between consecutive dispatches on the queue."""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
gaps = []
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0]
    dur[name].append(e - s)
    if prev_end is not None and s > prev_end:
        gaps.append(s - prev_end)
    prev_end = e if prev_end is None else max(prev_end, e)
tot = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
busy = sum(sum(v) for v in dur.values())
print(f"dispatches={len(rows)} span={tot/1e6:.2f} ms busy={busy/1e6:.2f} ms ({100*busy/tot:.1f}%)")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(f"  {k:45s} n={len(v):6d} mean={statistics.mean(v)/1e3:8.2f} us  median={statistics.median(v)/1e3:8.2f} us")
if gaps:
    print(f"gaps: n={len(gaps)} mean={statistics.mean(gaps)/1e3:.2f} us median={statistics.median(gaps)/1e3:.2f} us "
          f"p90={sorted(gaps)[int(0.9*len(gaps))]/1e3:.2f} us")
