"""Per-kernel means of rocprofv3 --pmc counter passes: for every pass directory given, the mean value per
dispatch of each counter, grouped by a short kernel name (template arguments kept, namespaces dropped).

  python scripts/pmc_table.py gpurun_out/pc1 gpurun_out/pc2 ...   -> a markdown table on stdout"""
import collections
import csv
import os
import re
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    per = collections.defaultdict(float)  # (dispatch, kernel, counter) -> summed value (over XCD/SE dims)
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, k, c), v in per.items():
        name = re.sub(r"\(anonymous namespace\)::|es_gemm::|es_panel::|void |\(.*$", "", k)[:70]
        vals[name][c].append(v)
counters = sorted({c for k in vals for c in vals[k]})
print("| kernel | n | " + " | ".join(counters) + " |")
print("|---|---:|" + "---:|" * len(counters))
for k in sorted(vals):
    n = max(len(v) for v in vals[k].values())
    cells = []
    for c in counters:
        v = vals[k].get(c)
        cells.append(f"{sum(v) / len(v):.4g}" if v else "")
    print(f"| `{k}` | {n} | " + " | ".join(cells) + " |")
