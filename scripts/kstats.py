"""Per-step summary of a rocprofv3 kernel_stats.csv: python scripts/kstats.py <csv> <steps profiled> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel ms/step {tot / steps / 1e6:.2f}")
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.2f} {int(r['Calls']) / steps:6.1f} "
          f"{float(r['AverageNs']) / 1e3:8.1f}  {r['Name'][:100]}")
