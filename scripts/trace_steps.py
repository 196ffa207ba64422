"""Per-step view of a bench.py rocprofv3 kernel trace (steps delimited by adam_ema_kernel): span, kernel
time, the time at least one kernel runs (busy) and the per-kernel totals of the chosen steps.
  python scripts/trace_steps.py <run_kernel_trace.csv> [first_step] [n_steps] [n_rows]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 3
nst = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ends = [i for i, r in enumerate(rows) if "adam_ema_kernel" in r["Kernel_Name"]]
lo, hi = ends[first - 1] + 1, ends[first - 1 + nst]
sel = rows[lo:hi + 1]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel)
busy, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = (int(sel[-1]["End_Timestamp"]) - int(rows[ends[first - 1]]["End_Timestamp"])) / 1e3 / nst
agg = collections.defaultdict(lambda: [0.0, 0])
for r in sel:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\((?!anon).*", "", name)[:60]
    g = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
    wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or "1"
    key = f"{name} [{int(g) // max(1, int(wg))}]" if g else name
    agg[key][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / nst
    agg[key][1] += 1 / nst
tot = sum(v[0] for v in agg.values())
print(f"steps {first}..{first + nst - 1}: span {span / 1e3:.3f} ms/step, kernels {tot / 1e3:.3f} ms, "
      f"busy {busy / 1e6 / nst:.3f} ms, launches {len(sel) / nst:.1f}")
for k, (us, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:int(sys.argv[4]) if len(sys.argv) > 4 else 45]:
    print(f"{us / 1e3:7.3f} ms {c:6.1f} x {us / c:8.1f} us  {k}")
