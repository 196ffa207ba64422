"""Phase timing of the single-pass attention backward (es_set_attn_bwd_variant 5: s_memtime stamps of workgroups
0 and 101) at the F1 shape: per phase, the median over heads of the slowest / fastest wave, in shader cycles.

  python scripts/attn_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

NAMES = ["top wait+barrier", "deltas+barrier", "phase1A", "K wait+barrier", "phase2A", "barrier", "phase1B+dKV",
         "barrier", "phase2B", "barrier"]


def main():
    lib = _lib.load()
    n, T, H = 512, 197, 6
    D = 64 * H
    torch.manual_seed(0)
    qkv = (torch.randn(n * T, 3 * D, device="cuda") * 0.5).bfloat16()
    o = torch.empty(n * T, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(n * H * T, device="cuda")
    delta = torch.empty(n * H * T, device="cuda")
    do = torch.randn(n * T, D, device="cuda").bfloat16()
    dqkv = torch.empty(n * T, 3 * D, device="cuda", dtype=torch.bfloat16)
    s = _lib.stream()
    call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 0.125, s)
    old = lib.es_set_attn_bwd_variant(5)
    for _ in range(3):
        call("es_attn_bwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), ptr(delta), ptr(do), D, ptr(dqkv), 3 * D, n, T, H,
             0.125, s)
    torch.cuda.synchronize()
    lib.es_set_attn_bwd_variant(old)
    st = np.zeros((2, 8, 16, 12), dtype=np.uint64)
    f = lib.es_attn_bwd_stamps
    f.argtypes = [ctypes.c_void_p]
    assert f(st.ctypes.data) == 0
    st = st.astype(np.int64)
    for wg in range(2):
        heads = [h for h in range(16) if st[wg, :, h, 9].min() > 0]
        t0 = st[wg, :, 0, 11].min()
        print(f"workgroup {[0, 101][wg]}: {len(heads)} heads, total {st[wg, :, heads[-1], 9].max() - t0} cycles")
        rows = []
        for k in range(10):
            prev = (st[wg, :, :, k - 1] if k else np.concatenate([st[wg, :, :1, 11], st[wg, :, :-1, 9]], axis=1))
            d = st[wg, :, :, k] - prev
            d = d[:, heads]
            rows.append((NAMES[k], int(np.median(d.max(axis=0))), int(np.median(d.min(axis=0)))))
        tot = sum(r[1] for r in rows)
        for name, mx, mn in rows:
            print(f"  {name:18s} max-wave {mx:7d}  min-wave {mn:7d}  ({100 * mx / tot:.0f}%)")


if __name__ == "__main__":
    main()
