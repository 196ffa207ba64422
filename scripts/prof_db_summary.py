"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite output) of a bench.py workload:
per-step wall / summed kernel time (steps delimited by the fused Adam + EMA launch) and the last
step's kernels by total time.
  python scripts/prof_db_summary.py <rocprof dir> <out.md> [title]"""
import collections
import glob
import re
import sqlite3
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else src
    db = glob.glob(src + "/**/*.db", recursive=True)[0]
    rows = sqlite3.connect(db).execute(
        "select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
    ad = [r for r in rows if "adam" in r[0]]
    bounds = [rows[0][1]] + [a[2] for a in ad]
    lines = [f"# {title}", "", "rocprofv3 --kernel-trace --stats; steps delimited by the Adam + EMA launch "
             "(step 0 = warmup, includes first-launch costs). Kernel time > wall time where kernels of the "
             "two branch streams / the weight-gradient side stream overlap.", "",
             "| step | wall ms | summed kernel ms | launches |", "|---:|---:|---:|---:|"]
    for s in range(len(ad)):
        seg = [r for r in rows if bounds[s] <= r[1] < bounds[s + 1]]
        lines.append(f"| {s} | {(bounds[s + 1] - bounds[s]) / 1e6:.1f} | {sum(r[2] - r[1] for r in seg) / 1e6:.1f} | "
                     f"{len(seg)} |")
    seg = [r for r in rows if bounds[-2] <= r[1] < bounds[-1]]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seg:
        n = re.sub(r"\(anonymous namespace\)::|es_gemm::", "", r[0])[:90].replace("|", "/")
        agg[n][0] += 1
        agg[n][1] += (r[2] - r[1]) / 1e6
    tot = sum(v[1] for v in agg.values())
    lines += ["", f"Last step by kernel ({tot:.1f} ms summed):", "", "| ms | % | launches | avg us | kernel |",
              "|---:|---:|---:|---:|---|"]
    for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
        lines.append(f"| {t:.2f} | {100 * t / tot:.1f} | {k} | {t / k * 1e3:.1f} | `{n}` |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:12]))


if __name__ == "__main__":
    main()
