"""Busy-time analysis of a rocprofv3 kernel trace: per-queue busy time, the union over queues (chip
busy), and the time two or more kernels ran together.  python scripts/trace_overlap.py <trace.csv> [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ev = []
per_q = {}
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
    per_q.setdefault(q, []).append((s, e))
    ev += [(s, 1), (e, -1)]
ev.sort()
busy = multi = 0
depth, last = 0, None
for t, d in ev:
    if last is not None and depth > 0:
        busy += t - last
        if depth > 1:
            multi += t - last
    depth += d
    last = t
span = max(e for _, e in sum(per_q.values(), [])) - min(s for s, _ in sum(per_q.values(), []))
print(f"span {span / 1e6 / steps:.2f} ms/step, chip busy {busy / 1e6 / steps:.2f}, two+ kernels together "
      f"{multi / 1e6 / steps:.2f}")
for q, iv in per_q.items():
    print(f"  queue {q}: {len(iv) / steps:.0f} kernels/step, {sum(e - s for s, e in iv) / 1e6 / steps:.2f} ms/step")
