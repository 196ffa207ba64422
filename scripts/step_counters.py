"""Per-kernel-family counters of ONE F1 step from scripts/gpu_step_counters.sh's rocprofv3 passes over bench.py
(the last of the 2 timed steps: the dispatches after the second-to-last adam_ema launch, up to and including
the last one; the bench's own extra single-stream steps come after the timed ones and are excluded by
taking the step that ends at the (warmup + steps)-th adam_ema dispatch).

  MFMA utilisation of a kernel  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x its duration x clock)
  step MFMA utilisation         = sum over the step's kernels of SQ_VALU_MFMA_BUSY_CYCLES
                                  / (1024 SIMDs x the step's wall time x clock)
  HBM bytes                     = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts a 128-B streaming read as 64 B,
                                  MI355X_MICROARCH.md §HBM) + WRITE_SIZE, KiB -> B
  clock                         = GRBM_GUI_ACTIVE / 8 XCDs / duration, per kernel (the effective clock the
                                  chip held); the step figure uses the busy-cycle-weighted mean of those, and
                                  the nominal 2.4 GHz as the lower bound of utilisation
  python scripts/step_counters.py gpurun_out r04   -> profiles/r04_step_counters.{md,json}"""
import collections
import csv
import json
import os
import re
import sys

root, tag = sys.argv[1], sys.argv[2]
WARMUP, STEPS = 1, 2
NSIMD, NOMINAL = 1024, 2.4e9


def rows(i):
    d = os.path.join(root, f"scnt{i}")
    cc = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    per = collections.defaultdict(float)
    meta = {}
    for r in cc:
        key = int(r["Dispatch_Id"])
        per[(key, r["Counter_Name"])] += float(r["Counter_Value"])
        meta[key] = r["Kernel_Name"]
    tr = {int(r["Dispatch_Id"]): (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
          for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))}
    return per, meta, tr


def family(name):
    n = name.lower()
    for key, fam in (("gemm_resid_ln", "projection + residual + LayerNorm 2 (fused)"),
                     ("gemm_panel", "NT GEMM (panel K=384)"), ("gemm_nt", "NT GEMM (tiled)"),
                     ("gemm_tn", "weight-gradient GEMM (TN)"), ("splitk_reduce", "split-K / bias reductions"),
                     ("reduce_partials", "split-K / bias reductions"), ("colsum", "split-K / bias reductions"),
                     ("attn", "attention"), ("layernorm", "LayerNorm"), ("ln_", "LayerNorm"),
                     ("adam", "Adam + EMA"), ("im2col", "patch gather / embedding"), ("embed", "patch gather / embedding")):
        if key in n:
            return fam
    return "other"


def step_window(meta, tr):
    ids = sorted(meta)
    adam = [i for i in ids if "adam_ema" in meta[i]]
    end = adam[WARMUP + STEPS - 1]
    start = adam[WARMUP + STEPS - 2]
    return [i for i in ids if start < i <= end]


out = {}
p1, m1, t1 = rows(1)
win = step_window(m1, t1)
wall = (max(t1[i][1] for i in win) - min(t1[i][0] for i in win)) * 1e-9
fam = collections.defaultdict(lambda: collections.defaultdict(float))
for i in win:
    f = family(m1[i])
    dur = (t1[i][1] - t1[i][0]) * 1e-9
    fam[f]["launches"] += 1
    fam[f]["kernel_s"] += dur
    fam[f]["mfma_busy"] += p1[(i, "SQ_VALU_MFMA_BUSY_CYCLES")]
    fam[f]["grbm"] += p1[(i, "GRBM_GUI_ACTIVE")]
    fam[f]["mfma_insts"] += p1[(i, "SQ_INSTS_MFMA")]
# bytes (the same step window by position: the passes dispatch the same kernel sequence)
for pi, cname in ((2, "FETCH_SIZE"), (3, "WRITE_SIZE")):
    pp, mm, tt = rows(pi)
    w2 = step_window(mm, tt)
    assert [family(mm[i]) for i in w2] == [family(m1[i]) for i in win], "passes dispatched different kernels"
    for i in w2:
        fam[family(mm[i])][cname] += pp[(i, cname)] * 1024
tot = collections.defaultdict(float)
lines = [f"# {tag}: step-level counters, F1 bench step (rocprofv3 --pmc over `bench.py --steps 2 --warmup 1`)", "",
         "One FixMatch ViT-S/16 step at configs[1] (B=64, mu=7), the second timed step; per kernel family. MFMA "
         "util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel time x effective clock GRBM_GUI_ACTIVE/8/time); "
         "HBM = 2 x FETCH_SIZE + WRITE_SIZE. Profiled passes run at a lower clock than the bench "
         "(MI355X_MICROARCH.md DVFS item 2).", "",
         "| family | launches | kernel ms | MFMA util (own time) | HBM GB | HBM TB/s (own time) |",
         "|---|---:|---:|---:|---:|---:|"]
for f, v in sorted(fam.items(), key=lambda kv: -kv[1]["kernel_s"]):
    clk = v["grbm"] / 8 / v["kernel_s"] if v["kernel_s"] else NOMINAL
    util = v["mfma_busy"] / (NSIMD * v["kernel_s"] * clk) if v["kernel_s"] else 0.0
    hbm = 2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]
    out[f] = {"launches": int(v["launches"]), "kernel_ms": v["kernel_s"] * 1e3, "mfma_util": util,
              "hbm_bytes": hbm, "hbm_tbs": hbm / v["kernel_s"] / 1e12 if v["kernel_s"] else 0.0, "clock_ghz": clk / 1e9}
    for k in ("mfma_busy", "grbm", "kernel_s", "mfma_insts"):
        tot[k] += v[k]
    tot["hbm"] += hbm
    lines.append(f"| {f} | {int(v['launches'])} | {v['kernel_s'] * 1e3:.2f} | {util:.3f} | {hbm / 1e9:.2f} | "
                 f"{out[f]['hbm_tbs']:.2f} |")
clk = tot["grbm"] / 8 / tot["kernel_s"]
step = {"wall_ms": wall * 1e3, "kernel_ms_sum": tot["kernel_s"] * 1e3, "mfma_busy_simd_cycles": tot["mfma_busy"],
        "mfma_util_effective_clock": tot["mfma_busy"] / (NSIMD * wall * clk), "effective_clock_ghz": clk / 1e9,
        "mfma_util_nominal_clock": tot["mfma_busy"] / (NSIMD * wall * NOMINAL), "hbm_bytes": tot["hbm"],
        "hbm_tbs": tot["hbm"] / wall / 1e12}
lines += ["", f"Step (profiled): wall {wall * 1e3:.2f} ms (two streams), kernel time {tot['kernel_s'] * 1e3:.2f} ms; "
          f"MFMA-busy SIMD-cycles {tot['mfma_busy']:.4g}; step MFMA utilisation "
          f"**{step['mfma_util_effective_clock']:.3f}** at the effective clock {clk / 1e9:.2f} GHz "
          f"({step['mfma_util_nominal_clock']:.3f} at the nominal 2.4 GHz); HBM {tot['hbm'] / 1e9:.2f} GB = "
          f"{step['hbm_tbs']:.2f} TB/s over the step."]
pdir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
import hashlib  # noqa: E402
_lib_so = os.path.join(os.path.dirname(pdir), "endoscopy-image-classification_amd", "endossl", "lib", "libendossl_hip.so")
res = {"tag": tag, "families": out, "step": step,
       "lib_sha256": hashlib.sha256(open(_lib_so, "rb").read()).hexdigest(),
       "source": "scripts/gpu_step_counters.sh (rocprofv3 --kernel-trace --pmc, 3 passes over bench.py)"}
json.dump(res, open(os.path.join(pdir, f"{tag}_step_counters.json"), "w"), indent=1)
open(os.path.join(pdir, f"{tag}_step_counters.md"), "w").write("\n".join(lines) + "\n")
