"""Embedding-backward microbenchmark at the F1 train shape (512 images x 197 tokens x 384):
python scripts/embed_bench.py [--iters 20]  (ENDOSSL_LIB selects the library for same-box A/B)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pad", type=int, default=0, help="row stride D + pad (1: the per-feature kernel)")
    args = ap.parse_args()
    n, T, D = 512, 197, 384
    ld = D + args.pad
    dx = torch.randn(n * T, ld, device="cuda")
    dpatch = torch.empty(n * (T - 1), D, device="cuda", dtype=torch.bfloat16)
    dpos = torch.empty(T * D, device="cuda")
    dcls = torch.empty(D, device="cuda")
    s = _lib.stream()
    f = lambda: call("es_embed_bwd", ptr(dx), ld, ptr(dpatch), D, ptr(dpos), ptr(dcls), n, T, D, 0, s)  # noqa: E731
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f()
        e0.record()
        for _ in range(args.iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / args.iters * 1e3)
    print(f"embed_bwd {sorted(ts)[2]:.1f} us (row stride {ld}; {os.environ.get('ENDOSSL_LIB', 'in-tree')})")


if __name__ == "__main__":
    main()
