"""SQ-counter ratios per kernel from rocprofv3 --pmc passes: python scripts/pmc_ratios.py <glob of run dirs>"""
import collections
import csv
import glob
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(\w+_kernel(<[^>]*>)?)", r["Kernel_Name"])
            if m:
                agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    d = {c: sum(x) / len(x) for c, x in v.items()}
    if "SQ_WAVE_CYCLES" not in d or "SQ_INSTS_MFMA" not in d or not d["SQ_INSTS_MFMA"]:
        continue
    wc = d["SQ_WAVE_CYCLES"]
    print(f"{k}: wait_any {d['SQ_WAIT_ANY'] / wc:.2f} wait_inst {d['SQ_WAIT_INST_ANY'] / wc:.2f} "
          f"active {d['SQ_ACTIVE_INST_ANY'] / wc:.2f} | VALU/MFMA {(d['SQ_INSTS_VALU'] - d['SQ_INSTS_MFMA']) / d['SQ_INSTS_MFMA']:.2f} "
          f"LDS/MFMA {d['SQ_INSTS_LDS'] / d['SQ_INSTS_MFMA']:.2f} bank_conflict/LDS "
          f"{d['SQ_LDS_BANK_CONFLICT'] / max(1, d['SQ_INSTS_LDS']):.2f} vmem_cyc {d.get('SQ_INST_CYCLES_VMEM', 0) / wc:.3f} mfma_busy/wave_cyc {d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / wc:.3f}")
