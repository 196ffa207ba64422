"""Per-launch HBM bytes of the roofline launch -- a block's weight gradients as one grouped split-K
launch (es_gemm_tn_big_grouped: gemm_tn_big_grouped_kernel + splitk_reduce_grouped_kernel) -- inside a
whole F1 step, from the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc_step.sh over bench.py.
FETCH_SIZE x2 (the gfx950 correction of MI355X_MICROARCH.md), KiB -> bytes.  Blocks 10..1 (the CU-share
sized launches; block 0's runs on the whole chip after the chain, the last block's is the K/V slice
alone).  Writes the entry bench.py reports as roofline.traffic into profiles/pmc_traffic.json.
  python scripts/pmc_layer_bytes.py gpurun_out [step] [tag]"""
import csv
import json
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
want = int(sys.argv[2]) if len(sys.argv) > 2 else 2
tag = sys.argv[3] if len(sys.argv) > 3 else "r05"
seqs = {}
for i, cname in ((1, "FETCH_SIZE"), (2, "WRITE_SIZE")):
    rows = sorted((r for r in csv.DictReader(open(f"{root}/pstep{i}/run_counter_collection.csv"))
                   if r["Counter_Name"] == cname), key=lambda r: int(r["Dispatch_Id"]))
    step, seq = 0, []
    for r in rows:
        if step == want:
            seq.append((r["Kernel_Name"], float(r["Counter_Value"]) * 1024))
        if "adam_ema" in r["Kernel_Name"]:
            step += 1
    seqs[cname] = seq
f, w = seqs["FETCH_SIZE"], seqs["WRITE_SIZE"]
assert [a[0] for a in f] == [b[0] for b in w], "the two passes dispatched different kernels"
sites, cur = [], None
for (name, fb), (_, wb) in zip(f, w):
    if "gemm_tn_big_grouped" in name:
        cur = {"kernel": 2 * fb + wb, "reduce": 0.0}
        sites.append(cur)
    elif cur is not None and "splitk_reduce_grouped" in name:
        cur["reduce"] += 2 * fb + wb
        cur = None
full = sites[1:-1]  # blocks 10..1
tot = [s["kernel"] + s["reduce"] for s in full]
M, D, Hd = 512 * 197, 384, 1536
alg = sum(2 * M * (a + b) + 4 * a * b + 4 * a for a, b in ((D, Hd), (Hd, D), (D, D), (3 * D, D)))
entry = {
    "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py (scripts/gpu_pmc_step.sh), step {want} "
              f"of the F1 run, {len(full)} grouped block launches (blocks 10..1)",
    "hbm_bytes_per_launch": int(round(statistics.median(tot))),
    "kernel_bytes": int(round(statistics.median(s["kernel"] for s in full))),
    "reduce_bytes": int(round(statistics.median(s["reduce"] for s in full))),
    "algorithmic_bytes_per_launch": alg,
    "ratio": round(statistics.median(tot) / alg, 4),
    "note": "per block: dY and X of fc2 / fc1 / proj / qkv bf16 once + fp32 weight and bias outputs; the rest are "
            "the split-K slabs written by the GEMM kernel and re-read by the reduction",
}
import hashlib  # noqa: E402
_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
entry["lib_sha256"] = hashlib.sha256(open(os.path.join(_root, "endoscopy-image-classification_amd", "endossl", "lib",
                                                       "libendossl_hip.so"), "rb").read()).hexdigest()
print(json.dumps(entry, indent=1))
p = os.path.join(_root, "profiles", "pmc_traffic.json")
d = json.load(open(p))
# the newest measurement first (bench.py reports the first entry that names the kernel); older ones kept as history
d["kernels"] = {f"es_gemm_tn_big_grouped block weight gradients in the F1 step ({tag})": entry,
                **{k: v for k, v in d["kernels"].items() if not k.endswith(f"({tag})")}}
json.dump(d, open(p, "w"), indent=1)
