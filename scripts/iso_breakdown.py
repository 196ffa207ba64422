"""Per-kernel time of the single-stream (isolated) steps at the end of a bench.py rocprofv3 trace:
bench.py runs its last 2 steps with the engine's second stream off, so these kernels ran alone.
  python scripts/iso_breakdown.py <run_kernel_trace.csv> [n_last_steps]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ends = [i for i, r in enumerate(rows) if "adam_ema_kernel" in r["Kernel_Name"]]
lo = ends[-nlast - 1] + 1
sel = rows[lo:ends[-1] + 1]
agg = collections.defaultdict(lambda: [0.0, 0])
for r in sel:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\((?!anon).*", "", name)[:70]
    g = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[name][0] += d / nlast
    agg[name][1] += 1 / nlast
tot = sum(v[0] for v in agg.values())
span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3 / nlast
print(f"isolated step: kernels {tot / 1e3:.2f} ms, span {span / 1e3:.2f} ms")
for k, (us, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"{us / 1e3:7.3f} ms {c:6.1f} x {us / c:8.1f} us  {k}")
