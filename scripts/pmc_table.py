"""Aggregate rocprofv3 --pmc passes (gpurun_out/sq*/run_counter_collection.csv) per (kernel, grid)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
agg = collections.OrderedDict()
for f in sorted(glob.glob(f"{root}/sq*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "es_gemm" not in r["Kernel_Name"] and "attn" not in r["Kernel_Name"] and "ln_" not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"].split("(")[0].replace("void ", "")[:48], r["Grid_Size"])
        agg.setdefault(k, collections.defaultdict(list))[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k)
    print("   ", ", ".join(f"{c}={sum(x) / len(x):.3g}" for c, x in v.items()))
