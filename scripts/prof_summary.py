"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into profiles/<tag>_*.

  python scripts/prof_summary.py gpurun_out/prof <tag> [steps_profiled | 0] [bench log of the profiled process]
(with the bench log: the line's live roofline span next to the trace's span of the same launches in the timed
steps -- the bench's warm-up steps, then its timed ones, are the first optimizer launches of the trace)
Writes <tag>_kernel_stats.csv (rocprofv3's own summary, copied) and <tag>_summary.md
(per-kernel ms/step, per-shape GEMM/attention breakdown from the trace)."""
import collections
import csv
import os
import re
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 and int(sys.argv[3]) > 0 else None  # default: optimizer launches
benchlog = sys.argv[4] if len(sys.argv) > 4 else None
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "profiles")
os.makedirs(out, exist_ok=True)
shutil.copy(os.path.join(src, "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
rows = list(csv.DictReader(open(os.path.join(src, "run_kernel_stats.csv"))))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
if steps is None:  # every step the bench runs (warm-up, timed, its probes) ends in one adam_ema launch
    steps = sum(int(r["Calls"]) for r in rows if "adam_ema_kernel(" in r["Name"]) or 7
lines = [f"# {tag}: rocprofv3 --kernel-trace --stats of `bench.py` (1x MI355X)", "",
         f"Total GPU kernel time / step: **{tot / 1e6 / steps:.2f} ms** (every kernel of the profiled process over its {steps} "
         "optimizer launches, so the bench's isolated-kernel and probe launches are included; one step's own kernel "
         "time is in the step-counter table)", "",
         "| ms/step | % | calls/step | avg us | kernel |", "|---:|---:|---:|---:|---|"]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    name = re.sub(r"\(anonymous namespace\)::|es_gemm::", "", r["Name"])[:110].replace("|", "/")
    lines.append(f"| {float(r['TotalDurationNs']) / 1e6 / steps:.3f} | {float(r['Percentage']):.1f} | "
                 f"{int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | `{name}` |")
tr = os.path.join(src, "run_kernel_trace.csv")
if os.path.exists(tr):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(tr)):
        m = re.search(r"(gemm_nt\w*<[^>]*>|gemm_tn_kernel|gemm_tn_big_grouped_kernel|gemm_tn_big_kernel|"
                      r"splitk_reduce_grouped_kernel|splitk_reduce_kernel|attn_\w+<\d+>)",
                      r["Kernel_Name"])
        if not m:
            continue
        k = (m.group(1), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    lines += ["", "Per launch shape (workgroups identify M,N):", "", "| ms/step | calls/step | avg us | kernel | grid |",
              "|---:|---:|---:|---|---:|"]
    for (n, g), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        lines.append(f"| {t / steps / 1e3:.3f} | {c / steps:.1f} | {t / c:.1f} | `{n}` | {g} |")
    # the roofline site as the bench times it: a 96-workgroup grouped launch's start to the end of the reduce
    # launch that follows it on the same queue
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r["Queue_Id"]].append(r)
    spans, kern = [], []
    for q in byq.values():
        for i, r in enumerate(q[:-1]):
            if ("tn_big_grouped" in r["Kernel_Name"] and int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) == 96
                    and "splitk_reduce_grouped" in q[i + 1]["Kernel_Name"]):
                spans.append((int(q[i + 1]["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                kern.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    site = (f" In this trace: {len(spans)} such launches, kernel {sum(kern) / len(kern):.1f} us on average, "
            f"kernel start to reduce end {sum(spans) / len(spans):.1f} us (the span the bench's `mean_launch_ms` "
            "times with kernel-stamped events).") if spans else ""
    if spans and benchlog and os.path.exists(benchlog):
        import json
        line = json.loads([x for x in open(benchlog) if x.startswith('{"metric')][-1])
        w, k = line["warmup"], line["steps"]
        # launches per optimizer step, in trace order (all queues): the timed steps are steps [w, w + k)
        bounds = [int(r["Start_Timestamp"]) for r in rows if "adam_ema_kernel(" in r["Kernel_Name"]]
        t0 = bounds[w - 1] if w > 0 else 0
        t1 = bounds[w + k - 1]
        per_step = collections.defaultdict(list)  # the timed steps' launches, by step, in start order
        for q in byq.values():
            for i, r in enumerate(q[:-1]):
                st = int(r["Start_Timestamp"])
                if ("tn_big_grouped" in r["Kernel_Name"] and int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) == 96
                        and "splitk_reduce_grouped" in q[i + 1]["Kernel_Name"] and t0 < st < t1):
                    step = sum(1 for x in bounds if x < st)
                    per_step[step].append((st, (int(q[i + 1]["End_Timestamp"]) - st) / 1e3,
                                           (int(r["End_Timestamp"]) - st) / 1e3))
        # each step's first such launch is the last block's (its K / V slice only, ~0.19 ms): the line times
        # blocks 10..1
        tspan = [sp for v in per_step.values() for _, sp, _ in sorted(v)[1:]]
        tkern = [kk for v in per_step.values() for _, _, kk in sorted(v)[1:]]
        rl = line["roofline"]
        site += (f" In the {k} timed steps of the same process, blocks 10..1 ({len(tspan)} launches): kernel start to "
                 f"reduce end {sum(tspan) / len(tspan):.1f} us (kernel alone {sum(tkern) / len(tkern):.1f} us) against "
                 f"the bench line's `mean_launch_ms` {rl['mean_launch_ms'] * 1e3:.1f} us over its {rl.get('launches')} "
                 f"launches: {rl['mean_launch_ms'] * 1e3 / (sum(tspan) / len(tspan)):.3f}x.")
    lines += ["", "The bench's roofline site (a block's four weight-gradient GEMMs, fc2 / fc1 / proj / qkv over "
              "M = 100,864 tokens) is the `gemm_tn_big_grouped_kernel` launch of 96 workgroups (24 tiles of 384 x 192 "
              "x 4 splits, 3/8 of the CUs, 11 per step: blocks 11..1, block 11's on its K / V slice alone) plus its `splitk_reduce_grouped_kernel`; the first block's "
              "launch (whole chip, the end of the backward) and the patch embedding's are other grid sizes above."
              + site + " Durations under the profiler run at lower clocks (MI355X_MICROARCH.md 'DVFS give-back' "
              "item 2)."]
    if benchlog and os.path.exists(benchlog):
        # the timed steps alone: every launch that starts after the warm-up's last optimizer launch and ends by the
        # last timed one (the process's allocations, warm-up, isolated-roofline and probe launches excluded)
        import json
        line = json.loads([x for x in open(benchlog) if x.startswith('{"metric')][-1])
        w, k = line["warmup"], line["steps"]
        bounds = [int(r["End_Timestamp"]) for r in rows if "adam_ema_kernel(" in r["Kernel_Name"]]
        t0, t1 = (bounds[w - 1] if w > 0 else 0), bounds[w + k - 1]
        inside = [r for r in rows if t0 < int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= t1]
        fills_in = sum(1 for r in inside if "FillFunctor" in r["Kernel_Name"])
        fills_all = sum(1 for r in rows if "FillFunctor" in r["Kernel_Name"])
        agg2 = collections.defaultdict(lambda: [0, 0.0])
        for r in inside:
            name = re.sub(r"\(anonymous namespace\)::|es_gemm::|void ", "", r["Kernel_Name"])
            name = re.sub(r"\((?!anon).*", "", name)[:90].replace("|", "/")
            agg2[name][0] += 1
            agg2[name][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        ktot = sum(v[1] for v in agg2.values())
        lines += ["", f"Inside the {k} timed steps alone ({len(inside) / k:.1f} launches / step, kernel time "
                  f"{ktot / k / 1e3:.2f} ms / step over two streams, wall {(t1 - t0) / 1e6 / k:.2f} ms / step under the "
                  f"profiler): torch `FillFunctor` launches inside the steps: **{fills_in}** (in the whole process: "
                  f"{fills_all}, all at allocation / warm-up outside `step()`).", "",
                  "| ms/step | calls/step | avg us | kernel |", "|---:|---:|---:|---|"]
        for n, (c, t) in sorted(agg2.items(), key=lambda x: -x[1][1])[:40]:
            lines.append(f"| {t / k / 1e3:.3f} | {c / k:.1f} | {t / c:.1f} | `{n}` |")
open(os.path.join(out, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:20]))
