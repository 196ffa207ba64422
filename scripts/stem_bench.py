"""Stem conv (3 -> 64, 7x7 / 2 / 3, NHWC fp32 images) forward and weight gradient at the S1 (120 x 384^2) and
P0 (16 x 224^2) shapes, the specialised kernels (es_set_stem_kernels(1)) vs the generic ones (0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402


def timed(fn, iters=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


lib = _lib.load()
s = _lib.stream()
for name, N, H in (("S1", 120, 384), ("P0", 16, 224)):
    Ho = H // 2
    x = torch.randn(N, H, H, 3, device="cuda")
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    y = torch.empty(N, Ho, Ho, 64, device="cuda")
    dy = torch.randn(N, Ho, Ho, 64, device="cuda")
    dw = torch.empty(64, 3, 7, 7, device="cuda")
    M = N * Ho * Ho
    splits = max(1, min(-(-M // 64), -(-2048 // lib.es_conv2d_dw_tiles(64, 3, 7, 7))))
    ws = torch.empty(lib.es_conv2d_bwd_weight_workspace(64, 3, 7, 7, splits), device="cuda")
    for stem in (0, 1):
        lib.es_set_stem_kernels(stem)
        f = timed(lambda: call("es_conv2d_fwd", ptr(x), N, H, H, 3, H * H * 3, H * 3, 3, 1, ptr(w), None, 64, 7, 7, 2, 3,
                               ptr(y), Ho * Ho * 64, Ho * 64, 64, 0, s))
        b = timed(lambda: call("es_conv2d_bwd_weight", ptr(x), N, H, H, 3, H * H * 3, H * 3, 3, 1, ptr(dy),
                               Ho * Ho * 64, Ho * 64, 64, 64, 7, 7, 2, 3, splits, ptr(ws), ptr(dw), 0, s))
        print(f"{name} stem_kernels={stem}: fwd {f * 1e3:.1f} us, weight gradient {b * 1e3:.1f} us (splits {splits})",
              flush=True)
    lib.es_set_stem_kernels(1)
