"""Append the roofline kernel's per-phase average duration (from a rocprofv3 kernel trace of
`bench.py --steps 5 --warmup 2`) to profiles/<tag>_summary.md, beside bench.py's own HIP-event figures.

  python scripts/roofline_phases.py gpurun_out/prof_f1 <tag> <bench json line file>
Steps are delimited by the Adam/EMA sweep (adam_ema_kernel): 2 warm-up, 5 timed, 2 isolated."""
import collections
import csv
import json
import os
import sys

src, tag, bench = sys.argv[1], sys.argv[2], sys.argv[3]
kern = sys.argv[4] if len(sys.argv) > 4 else "gemm_nt_kernel<7, 32, 2>"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rows = sorted(csv.DictReader(open(os.path.join(src, "run_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
ends = [int(r["End_Timestamp"]) for r in rows if "adam_ema_kernel" in r["Kernel_Name"]]
b = json.loads([ln for ln in open(bench) if ln.startswith("{")][-1])["roofline"]


# the full-M launches only (the last block's CLS-row GEMMs use the same kernel on a small grid):
# the kernel's most frequent grid size
grids = collections.Counter(r.get("Grid_Size_X", r.get("Grid_Size", "")) for r in rows if kern in r["Kernel_Name"])
main_grid = grids.most_common(1)[0][0]


def avg(a, z):
    lo = ends[a - 1] if a > 0 else 0
    hi = ends[z]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
         if kern in r["Kernel_Name"] and lo < int(r["Start_Timestamp"]) <= hi
         and r.get("Grid_Size_X", r.get("Grid_Size", "")) == main_grid]
    return sum(d) / len(d) / 1e3, len(d)


t, nt = avg(2, 6)
i, ni = avg(7, 8)
txt = f"""

## Roofline kernel (`{kern}`: {b['kernel']}) by phase

Steps are delimited by the Adam/EMA sweep in the trace (2 warm-up, 5 timed, 2 isolated).

| phase | dispatches | avg us | bench.py's HIP-event figure (same config, separate process) |
|---|---:|---:|---|
| timed steps (weak forward co-running on the second stream) | {nt} | {t:.1f} | live `mean_launch_ms` {b['mean_launch_ms']:.3f} ms |
| isolated steps (`ENDOSSL_OVERLAP=0`) | {ni} | {i:.1f} | `isolated.mean_launch_ms` {b['isolated']['mean_launch_ms']:.3f} ms |
"""
open(os.path.join(root, "profiles", f"{tag}_summary.md"), "a").write(txt)
print(txt)
