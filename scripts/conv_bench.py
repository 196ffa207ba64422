"""Conv kernel microbenchmark over Conformer-Ti CNN-branch shapes (SemiFormer S1: 360 images).
  python scripts/conv_bench.py [--n 360]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

# (name, H, Cin, Cout, k, s, p)
SHAPES = [("s1_conv1_64to16", 56, 64, 16, 1, 1, 0), ("s1_conv2_16to16_3x3", 56, 16, 16, 3, 1, 1),
          ("s1_conv3_16to64", 56, 16, 64, 1, 1, 0), ("s1_res_64to64", 56, 64, 64, 1, 1, 0),
          ("s2_res_64to128_s2", 56, 64, 128, 1, 2, 0), ("s2_conv2_32to32_3x3", 28, 32, 32, 3, 1, 1),
          ("s3_conv2_64to64_3x3", 14, 64, 64, 3, 1, 1), ("s3_conv3_64to256", 14, 64, 256, 1, 1, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=360)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    _lib.load()
    s = _lib.stream()
    dev = "cuda"
    for name, H, Cin, Cout, k, st, p in SHAPES:
        N = a.n
        Ho = (H + 2 * p - k) // st + 1
        x = torch.randn(N, H, H, Cin, device=dev)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.1
        y = torch.empty(N, Ho, Ho, Cout, device=dev)
        dx = torch.empty_like(x)
        M = N * Ho * Ho
        flops = 2.0 * M * Cout * Cin * k * k
        splits = max(1, min(-(-M // 64), -(-2048 // _lib.load().es_conv2d_dw_tiles(Cout, Cin, k, k))))
        ws = torch.empty(_lib.load().es_conv2d_bwd_weight_workspace(Cout, Cin, k, k, splits), device=dev)
        dw = torch.empty_like(w)
        ops = {
            "fwd": lambda: call("es_conv2d_fwd", ptr(x), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(w), None,
                                Cout, k, k, st, p, ptr(y), Ho * Ho * Cout, Ho * Cout, Cout, 0, s),
            "dx": lambda: call("es_conv2d_bwd_data", ptr(y), Ho * Ho * Cout, Ho * Cout, Cout, ptr(w), N, H, H, Cin, Cout,
                               k, k, st, p, ptr(dx), H * H * Cin, H * Cin, Cin, 1, 0, s),
            "dw": lambda: call("es_conv2d_bwd_weight", ptr(x), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(y),
                               Ho * Ho * Cout, Ho * Cout, Cout, Cout, k, k, st, p, splits, ptr(ws), ptr(dw), 0, s),
        }
        res = {}
        for op, fn in ops.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / a.iters
            res[op] = f"{t * 1e3:8.1f}us {flops / t / 1e9:6.1f}TF"
        print(f"{name:24s} M={M:8d} GF={flops / 1e9:6.2f}  " + "  ".join(f"{k}:{v}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
