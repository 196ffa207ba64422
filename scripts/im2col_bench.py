"""uint8 patch gather at the F1 unlabeled batch (448 x 3 x 224^2): the LDS band kernel (16-B aligned pixels)
vs the element-wise gather (the same pixels at an 8-B offset), median ms.  python scripts/im2col_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

n, S = 448, 224
u8 = torch.randint(0, 256, (n * 3 * S * S + 16,), dtype=torch.uint8, device="cuda")
out = torch.empty(n * 196, 768, dtype=torch.bfloat16, device="cuda")
s = _lib.stream()
mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
res = {}
for name, off in (("band", 0), ("elementwise", 8), ("band", 0), ("elementwise", 8)):
    f = lambda: call("es_patch_im2col_u8", ptr(u8) + off, *mean, *std, ptr(out), n, S, 16, s)  # noqa: E731
    f()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    res.setdefault(name, []).append(round(sorted(ts)[10], 4))
byts = n * 3 * S * S + n * 196 * 768 * 2
print({k: (v, f"{byts / min(v) / 1e9:.2f} TB/s") for k, v in res.items()})
