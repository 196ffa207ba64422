"""Per-step stream busy times from a rocprofv3 kernel trace: steps delimited by the Adam/EMA sweep.
  python scripts/step_timeline.py <trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ends = [int(r["End_Timestamp"]) for r in rows if "adam_ema_kernel" in r["Kernel_Name"]]
prev = int(rows[0]["Start_Timestamp"])
for k, e in enumerate(ends):
    ks = [r for r in rows if prev < int(r["Start_Timestamp"]) <= e]
    per_q = {}
    for r in ks:
        per_q.setdefault(r["Queue_Id"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    ev = sorted([(s, 1) for v in per_q.values() for s, _ in v] + [(t, -1) for v in per_q.values() for _, t in v])
    busy = two = 0
    d, last = 0, None
    for t, x in ev:
        if last is not None and d > 0:
            busy += t - last
            if d > 1:
                two += t - last
        d += x
        last = t
    q = "  ".join(f"q{qq}: {sum(b - a for a, b in v) / 1e6:6.2f} ms ({len(v)} k)" for qq, v in sorted(per_q.items()))
    first = min(a for v in per_q.values() for a, _ in v)
    print(f"step {k}: span {(e - first) / 1e6:6.2f} ms  busy {busy / 1e6:6.2f}  2+ {two / 1e6:6.2f}  {q}")
    prev = e
