"""Add the roofline kernel's HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; scripts/gpu_pmc_fc1.sh) to profiles/pmc_traffic.json.

  python scripts/pmc_to_traffic.py <kernel substring> <entry name> <note>
FETCH_SIZE is doubled (MI355X_MICROARCH.md §HBM: gfx950 counts half of 16-B/lane streaming reads);
the 3rd dispatch of the kernel is used (1st = warm-up)."""
import csv
import json
import os
import sys

sub, entry, note = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(d, name):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(root, "gpurun_out", d,
                                                                                "run_counter_collection.csv")))
            if sub in r["Kernel_Name"] and r["Counter_Name"] == name]
    return vals[2] if len(vals) > 2 else vals[-1]


fk, wk = counter("fc1pmc1", "FETCH_SIZE"), counter("fc1pmc2", "WRITE_SIZE")
p = os.path.join(root, "profiles", "pmc_traffic.json")
d = json.load(open(p))
fb, wb = int(fk * 1024 * 2), int(wk * 1024)
d["kernels"][entry] = {"fetch_kib_raw": fk, "write_kib_raw": wk, "fetch_bytes": fb, "write_bytes": wb,
                       "hbm_bytes_per_launch": fb + wb, "algorithmic_bytes_per_launch": 698357760, "note": note}
json.dump(d, open(p, "w"), indent=1)
print(entry, fb + wb)
