"""Per-launch HBM bytes of the roofline site (the fc1 weight gradient) inside a whole F1 step, from
the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc_step.sh over bench.py.  The weight gradients
run on the engine's side stream in the order fc2, fc1, proj, qkv per block (after the last block's
K/V site); a site = its gemm_tn_big dispatch + the split-K reduction + the bias-partials reduction.
FETCH_SIZE x2 (the gfx950 correction of MI355X_MICROARCH.md), KiB -> bytes.  Writes the entry that
bench.py reports as roofline.traffic into profiles/pmc_traffic.json.
  python scripts/pmc_site_bytes.py gpurun_out [step]"""
import csv
import json
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
want = int(sys.argv[2]) if len(sys.argv) > 2 else 2
seqs = {}
for i, cname in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
    rows = sorted((r for r in csv.DictReader(open(f"{root}/pstep{i}/run_counter_collection.csv"))
                   if r["Counter_Name"] == cname), key=lambda r: int(r["Dispatch_Id"]))
    step, seq = 0, []
    for r in rows:
        if step == want:
            seq.append((r["Kernel_Name"], r["Queue_Id"], float(r["Counter_Value"]) * 1024))
        if "adam_ema" in r["Kernel_Name"]:
            step += 1
    seqs[cname] = seq
f, w = seqs["FETCH_SIZE"], seqs["WRITE_SIZE"]
assert [a[0] for a in f] == [b[0] for b in w], "the two passes dispatched different kernels"
q_side = next(a[1] for a in f if "gemm_tn_big" in a[0])
sites, cur = [], None
for (name, q, fb), (_, _, wb) in zip(f, w):
    if q != q_side:
        continue
    if "gemm_tn_big" in name:
        cur = {"kernel": 2 * fb + wb, "reduce": 0.0}
        sites.append(cur)
    elif cur is not None and ("splitk_reduce" in name or "reduce_partials" in name):
        cur["reduce"] += 2 * fb + wb
fc1 = [s for k, s in enumerate(sites[1:]) if k % 4 == 1]  # sites[0]: the last block's K/V weight gradient
tot = [s["kernel"] + s["reduce"] for s in fc1]
entry = {
    "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py (scripts/gpu_pmc_step.sh), step {want} "
              f"of the F1 run, {len(fc1)} fc1 weight-gradient sites (the 2nd of each block's four side-stream sites)",
    "hbm_bytes_per_launch": int(round(statistics.mean(tot))),
    "kernel_bytes": int(round(statistics.mean(s["kernel"] for s in fc1))),
    "reduce_bytes": int(round(statistics.mean(s["reduce"] for s in fc1))),
    "algorithmic_bytes_per_launch": 389_700_000,
    "note": "dY (310 MB) and X (77 MB) bf16 once + fp32 out; the rest are the split-K slabs written by the "
            "TN kernel and re-read by the reduction",
}
print(json.dumps(entry, indent=1))
p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
d = json.load(open(p))
d["kernels"] = {"es_gemm_tn fc1_wgrad in the F1 step (r02)": entry,
                **{k: v for k, v in d["kernels"].items() if "in the F1 step" not in k}}
json.dump(d, open(p, "w"), indent=1)
