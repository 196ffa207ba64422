"""Per-queue kernel breakdown of a rocprofv3 kernel trace: python scripts/queue_stats.py <trace.csv> <steps> [n]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 15
agg = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0]))
for r in rows:
    q = r.get("Queue_Id") or "0"
    name = r["Kernel_Name"]
    m = re.search(r"(\w+_kernel(<[^>]*>)?)", name)
    key = (m.group(1) if m else name[:40], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[q][key][0] += d
    agg[q][key][1] += 1
for q, kk in agg.items():
    tot = sum(v[0] for v in kk.values())
    print(f"queue {q}: {tot / steps / 1e6:.2f} ms/step")
    for k, v in sorted(kk.items(), key=lambda x: -x[1][0])[:n]:
        print(f"  {v[0] / steps / 1e6:7.2f} ms {v[1] / steps:5.1f}/step {v[0] / v[1] / 1e3:7.1f} us  {k[0]} grid={k[1]}")
