"""Kernel breakdown of selected steps (delimited by the Adam/EMA sweep) of a rocprofv3 kernel trace.
  python scripts/step_kernels.py <trace.csv> <first step> <last step> [n]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
a, b = int(sys.argv[2]), int(sys.argv[3])
n = int(sys.argv[4]) if len(sys.argv) > 4 else 30
ends = [int(r["End_Timestamp"]) for r in rows if "adam_ema_kernel" in r["Kernel_Name"]]
lo = ends[a - 1] if a > 0 else 0
hi = ends[b]
agg = collections.defaultdict(lambda: [0, 0])
tot = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if not (lo < s <= hi):
        continue
    m = re.search(r"(\w+_kernel(<[^>]*>)?)", r["Kernel_Name"])
    key = (m.group(1) if m else r["Kernel_Name"][:50], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
    agg[key][0] += e - s
    agg[key][1] += 1
    tot += e - s
steps = b - a + 1
print(f"kernel time {tot / steps / 1e6:.2f} ms/step over steps {a}..{b}")
for k, v in sorted(agg.items(), key=lambda x: -x[1][0])[:n]:
    print(f"  {v[0] / steps / 1e6:7.3f} ms {v[1] / steps:5.1f}/step {v[0] / v[1] / 1e3:7.1f} us  {k[0]} grid={k[1]}")
