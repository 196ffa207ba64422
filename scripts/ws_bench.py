"""The weight-stationary K = 384 NT GEMM (es_gemm_nt variant 12) against the per-shape default kernels at the
F1 shapes: outputs compared bit for bit, then timed in interleaved rounds (median), random operands.

  python scripts/ws_bench.py [--rounds 5] [--iters 20] [--only qkv_fwd,fc1_fwd]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

M_T, M_W = 512 * 197, 448 * 197
D, HD = 384, 1536
# (name, epi, M, N): K = 384 throughout
SHAPES = [("qkv_fwd", 0, M_T, 3 * D), ("qkv_fwd_weak", 0, M_W, 3 * D), ("fc1_fwd", 7, M_T, HD),
          ("fc1_fwd_weak", 6, M_W, HD), ("proj_dgrad", 0, M_T, D), ("fc1_gelu", 1, M_T, HD), ("proj_f32", 4, M_T, D)]
K = 384


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--base", type=int, default=-1, help="the variant to compare with (-1: the per-shape default)")
    args = ap.parse_args()
    lib = _lib.load()
    lib.es_set_gemm_variant.restype = _lib.I
    lib.es_set_gemm_variant.argtypes = [_lib.I]
    dev = "cuda"
    torch.manual_seed(0)
    s = _lib.stream()
    Mp = (M_T + 255) // 256 * 256
    A = torch.randn(Mp, K, device=dev).bfloat16()
    A[M_T:] = 0
    Bw = (torch.randn(HD, K, device=dev) * 0.05).bfloat16()
    bias = torch.randn(HD, device=dev) * 0.1
    outs = {v: (torch.empty(Mp, HD, device=dev), torch.empty(Mp, HD, device=dev, dtype=torch.bfloat16))
            for v in (args.base, 12)}
    only = set(args.only.split(",")) if args.only else None
    res = {}
    for name, epi, M, N in SHAPES:
        if only and name not in only:
            continue
        f32 = epi == 4

        def run(v, stream=None):
            C, C2 = outs[v]
            lib.es_set_gemm_variant(v)
            call("es_gemm_nt", epi, ptr(A), K, ptr(Bw), K, ptr(bias), ptr(C), N, ptr(C2) if epi in (1, 7) else None,
                 None, 0, M, N, K, 0, stream if stream is not None else s)

        def view(v, which):  # the [M, N] output as written (ldc = N)
            t = outs[v][which]
            if which == 0 and not f32:
                t = t.view(torch.bfloat16)
            return t.view(-1)[:M * N].view(M, N)

        # correctness: bit-identical outputs
        for v in (args.base, 12):
            outs[v][0].zero_()
            outs[v][1].zero_()
            run(v)
        torch.cuda.synchronize()
        same = bool(torch.equal(view(args.base, 0), view(12, 0)))
        if epi in (1, 7):
            same = same and bool(torch.equal(view(args.base, 1), view(12, 1)))
        times = {args.base: [], 12: []}
        for _ in range(args.rounds):
            for v in (args.base, 12):
                run(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.iters)
        row = {"bit_identical": same}
        for v in (args.base, 12):
            t = sorted(times[v])[len(times[v]) // 2]
            row[f"v{v}_us"] = round(t * 1000, 1)
        res[name] = row
        print(name, json.dumps(row), flush=True)
    if os.environ.get("ENDOSSL_WS_PROBE") == "7":  # per-step stamps of workgroup 0 (waves 0 and 4), last launch
        import ctypes
        buf = (ctypes.c_ulonglong * 1024)()
        lib.endossl_ws_debug_stamps(buf, 1024)
        st = [list(buf[i * 8:(i + 1) * 8]) for i in range(128)]
        for half, name in ((0, "wave0"), (1, "wave4")):
            rows = [r for r in st[half * 64:(half + 1) * 64] if r[0]]
            for i, r in enumerate(rows[:16]):
                # k: 7 top start, 0 after barrier, 1 after DMA issue, 2 after MFMA half 0, 3 after 2nd part,
                # 4 after 3rd part, 5 after last epilogue, 6 after tail
                print(name, i, "top-wait", r[0] - r[7], "dma", r[1] - r[0], "mfma0", r[2] - r[1], "part2", r[3] - r[2],
                      "part3", r[4] - r[3], "epi1", r[5] - r[4], "tail", r[6] - r[5],
                      "step", (rows[i + 1][7] - r[7]) if i + 1 < len(rows) else 0)
    lib.es_set_gemm_variant(-1)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "ws_bench.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
