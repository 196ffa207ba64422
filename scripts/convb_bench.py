"""bf16 conv kernels (csrc/conv_bf16.hip) in isolation over the Conformer-B/384 CNN-branch shapes
(SemiFormer S1: B=8, mu=7 -> 120 images).  Per shape and pass: HIP-event time of one launch
(+ its reduce for dW), algorithmic TFLOP/s (2 Cout Cin k^2 per output pixel) and GB/s of the
algorithmic bytes (fp32 maps read / written once, bf16 weights).
  python scripts/convb_bench.py [--n 120] [--iters 5]
  --bnin: bf16 maps, the shapes whose input is a BatchNorm + ReLU output (conv2 / conv3 of the ConvBlocks), each
  forward (with the next BatchNorm's statistics) and weight gradient timed plain and with the BatchNorm applied
  by the gather (es_conv2d_*_bf16_bnin_ex), interleaved"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

# (name, H (input), Cin, Cout, k, s, p)
SHAPES = [("st1_conv1_256to64", 96, 256, 64, 1, 1, 0), ("st1_conv2_64_3x3", 96, 64, 64, 3, 1, 1),
          ("st1_conv3_64to256", 96, 64, 256, 1, 1, 0), ("st2_conv1_512to128", 48, 512, 128, 1, 1, 0),
          ("st2_conv2_128_3x3", 48, 128, 128, 3, 1, 1), ("st2_conv3_128to512", 48, 128, 512, 1, 1, 0),
          ("st3_conv2_256_3x3", 24, 256, 256, 3, 1, 1), ("st3_conv3_256to1024", 24, 256, 1024, 1, 1, 0),
          ("patch_64to768_k4s4", 96, 64, 768, 4, 4, 0), ("st2_res_256to512_s2", 96, 256, 512, 1, 2, 0),
          ("fcu_up_768to64", 24, 768, 64, 1, 1, 0)]

# P0: timm resnet18 at 224^2 (B = 32 labeled images): every bf16 conv shape of the trunk
P0_SHAPES = [("l1_3x3_64", 56, 64, 64, 3, 1, 1), ("l2_3x3_64to128_s2", 56, 64, 128, 3, 2, 1),
             ("l2_3x3_128", 28, 128, 128, 3, 1, 1), ("l2_ds_64to128_s2", 56, 64, 128, 1, 2, 0),
             ("l3_3x3_128to256_s2", 28, 128, 256, 3, 2, 1), ("l3_3x3_256", 14, 256, 256, 3, 1, 1),
             ("l3_ds_128to256_s2", 28, 128, 256, 1, 2, 0), ("l4_3x3_256to512_s2", 14, 256, 512, 3, 2, 1),
             ("l4_3x3_512", 7, 512, 512, 3, 1, 1), ("l4_ds_256to512_s2", 14, 256, 512, 1, 2, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=120)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--bnin", action="store_true")
    ap.add_argument("--all-shapes", action="store_true", help="--bnin: every shape, not only conv2 / conv3")
    ap.add_argument("--p0", action="store_true", help="--bnin: the ResNet-18 (P0, n = 32) shapes instead")
    ap.add_argument("--f32maps", action="store_true", help="--bnin: fp32 activation / gradient maps (flags 0)")
    ap.add_argument("--ring", type=int, default=None, help="es_set_conv_ring first (0 = the register-staged gather)")
    ap.add_argument("--dwbuf", type=int, default=None, help="es_set_conv_dw_buf first (0 = the branchy weight gradient)")
    a = ap.parse_args()
    if a.bnin:
        return bnin_main(a)
    lib = _lib.load()
    s = _lib.stream()
    dev = "cuda"
    out = []
    for name, H, Cin, Cout, k, st, p in SHAPES:
        N = a.n
        Ho = (H + 2 * p - k) // st + 1
        M = N * Ho * Ho
        x = torch.randn(N, H, H, Cin, device=dev)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        y = torch.empty(N, Ho, Ho, Cout, device=dev)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        n = Cout * Cin * k * k
        wp = torch.empty(n, dtype=torch.bfloat16, device=dev)
        wt = torch.empty(n, dtype=torch.bfloat16, device=dev)
        dw = torch.empty_like(w)
        ws = torch.empty(lib.es_conv2d_bwd_weight_bf16_workspace(M, Cout, Cin, k, k, 0), device=dev)
        call("es_conv2d_pack_bf16", ptr(w), Cout, Cin, k, k, ptr(wp), ptr(wt), s)
        xs = (H * H * Cin, H * Cin, Cin, 1)
        ys = (Ho * Ho * Cout, Ho * Cout, Cout)

        def fwd():
            call("es_conv2d_fwd_bf16", ptr(x), N, H, H, Cin, *xs, ptr(wp), None, Cout, k, k, st, p, ptr(y), *ys, 0, s)

        def dgrad():
            call("es_conv2d_bwd_data_bf16", ptr(dy), *ys, ptr(wt), N, H, H, Cin, Cout, k, k, st, p, ptr(dx), *xs, 0, s)

        def wgrad():
            call("es_conv2d_bwd_weight_bf16", ptr(x), N, H, H, Cin, *xs, ptr(dy), *ys, Cout, k, k, st, p, 0, ptr(ws),
                 ptr(dw), 0, s)

        flop = 2.0 * M * Cout * Cin * k * k
        xb, yb = 4.0 * N * H * H * Cin, 4.0 * M * Cout
        rec = {"shape": name, "M": M, "GFLOP": round(flop / 1e9, 1)}
        for pas, fn, byts in (("fwd", fwd, xb + yb), ("dgrad", dgrad, xb + yb), ("wgrad", wgrad, xb + yb)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(a.iters):
                e0.record(torch.cuda.current_stream())
                fn()
                e1.record(torch.cuda.current_stream())
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = sorted(ts)[len(ts) // 2] * 1e-3
            rec[pas] = {"us": round(t * 1e6, 1), "TFLOPs": round(flop / t / 1e12, 1), "GBs": round(byts / t / 1e9)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del x, y, dy, dx, ws
        torch.cuda.empty_cache()
    tot = {p: sum(r[p]["us"] for r in out) for p in ("fwd", "dgrad", "wgrad")}
    print(json.dumps({"total_us": tot}))


def bnin_main(a):
    lib = _lib.load()
    if a.ring is not None:
        lib.es_set_conv_ring(a.ring)
    if a.dwbuf is not None:
        lib.es_set_conv_dw_buf(a.dwbuf)
    s = _lib.stream()
    dev = "cuda"
    res = {}
    for name, H, Cin, Cout, k, st, p in (P0_SHAPES if a.p0 else SHAPES):
        if not (a.all_shapes or a.p0) and "conv2" not in name and "conv3" not in name:
            continue
        N = 32 if a.p0 else a.n
        Ho = (H + 2 * p - k) // st + 1
        M = N * Ho * Ho
        mdt = torch.float32 if a.f32maps else torch.bfloat16
        fl = 0 if a.f32maps else 3
        x = torch.randn(N, H, H, Cin, device=dev).to(mdt)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        y = torch.empty(N, Ho, Ho, Cout, device=dev, dtype=mdt)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        mean, rstd = torch.randn(Cin, device=dev) * 0.1, torch.rand(Cin, device=dev) + 0.5
        gam, bet = torch.rand(Cin, device=dev) + 0.5, torch.randn(Cin, device=dev) * 0.1
        n = Cout * Cin * k * k
        wp = torch.empty(n, dtype=torch.bfloat16, device=dev)
        wt = torch.empty(n, dtype=torch.bfloat16, device=dev)
        dw = torch.empty_like(w)
        ws = torch.empty(lib.es_conv2d_bwd_weight_bf16_workspace(M, Cout, Cin, k, k, 0), device=dev)
        part = torch.empty(lib.es_conv2d_bnstats_size(M, Cout), device=dev)
        call("es_conv2d_pack_bf16", ptr(w), Cout, Cin, k, k, ptr(wp), ptr(wt), s)
        xs = (H * H * Cin, H * Cin, Cin, 1)
        ys = (Ho * Ho * Cout, Ho * Cout, Cout)
        bn = (ptr(mean), ptr(rstd), ptr(gam), ptr(bet))
        fns = {
            "fwd": lambda: call("es_conv2d_fwd_bf16_ex", ptr(x), N, H, H, Cin, *xs, ptr(wp), None, Cout, k, k, st, p,
                                ptr(y), *ys, 0, ptr(part), fl, s),
            "fwd_bnin": lambda: call("es_conv2d_fwd_bf16_bnin_ex", ptr(x), N, H, H, Cin, *xs, ptr(wp), None, Cout, k, k,
                                     st, p, ptr(y), *ys, 0, ptr(part), fl, *bn, s),
            "dgrad": lambda: call("es_conv2d_bwd_data_bf16_ex", ptr(dy), *ys, ptr(wt), N, H, H, Cin, Cout, k, k, st, p,
                                  ptr(dx), *xs, 0, fl, s),
            "wgrad": lambda: call("es_conv2d_bwd_weight_bf16_ex", ptr(x), N, H, H, Cin, *xs, ptr(dy), *ys, Cout, k, k,
                                  st, p, 0, ptr(ws), ptr(dw), 0, fl, s),
            "wgrad_bnin": lambda: call("es_conv2d_bwd_weight_bf16_bnin_ex", ptr(x), N, H, H, Cin, *xs, ptr(dy), *ys,
                                       Cout, k, k, st, p, 0, ptr(ws), ptr(dw), 0, fl, *bn, s),
        }
        ts = {kk: [] for kk in fns}
        for kk, fn in fns.items():
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.iters):
            for kk, fn in fns.items():
                e0.record(torch.cuda.current_stream())
                fn()
                e1.record(torch.cuda.current_stream())
                e1.synchronize()
                ts[kk].append(e0.elapsed_time(e1) * 1e3)
        res[name] = {kk: round(sorted(v)[len(v) // 2], 1) for kk, v in ts.items()}
        print(name, json.dumps(res[name]), flush=True)
        del x, y, dy, dx, ws
        torch.cuda.empty_cache()
    tot = {kk: round(sum(r[kk] for r in res.values()), 1) for kk in ("fwd", "fwd_bnin", "dgrad", "wgrad", "wgrad_bnin")}
    print(json.dumps({"total_us": tot}), flush=True)


if __name__ == "__main__":
    main()
