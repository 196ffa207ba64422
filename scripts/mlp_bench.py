"""Fused inference MLP (es_mlp_fwd_infer) vs the two GEMMs it replaces, at the F1 weak-forward shape
(M = 448 x 197 tokens, D = 384, Hd = 1536).  python scripts/mlp_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402


def timed(fn, iters=10, rounds=5):
    fn()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return sorted(ts)[len(ts) // 2]


def main():
    M, D, Hd = 448 * 197, 384, 1536
    Mp = (M + 255) // 256 * 256
    s = _lib.stream()
    h = torch.randn(Mp, D, device="cuda").bfloat16()
    W1 = (torch.randn(Hd, D, device="cuda") * 0.05).bfloat16()
    W2 = (torch.randn(D, Hd, device="cuda") * 0.025).bfloat16()
    b1, b2 = torch.randn(Hd, device="cuda"), torch.randn(D, device="cuda")
    resid = torch.randn(Mp, D, device="cuda")
    out = torch.empty(Mp, D, device="cuda")
    act = torch.empty(Mp, Hd, device="cuda", dtype=torch.bfloat16)
    W2c = W2.view(D, Hd // 32, 32).permute(1, 0, 2).contiguous()
    fused = timed(lambda: call("es_mlp_fwd_infer", ptr(h), D, ptr(W1), ptr(b1), ptr(W2c), ptr(b2), ptr(resid), D,
                               ptr(out), D, M, D, Hd, s))
    fc1 = timed(lambda: call("es_gemm_nt", 6, ptr(h), D, ptr(W1), D, ptr(b1), ptr(act), Hd, None, None, 0, M, Hd, D, 0,
                             s))
    fc2 = timed(lambda: call("es_gemm_nt", 2, ptr(act), Hd, ptr(W2), Hd, ptr(b2), ptr(out), D, None, ptr(resid), D, M,
                             D, Hd, 0, s))
    fl = 2 * 2.0 * M * D * Hd
    print(json.dumps({"fused_ms": round(fused, 4), "fused_tflops": round(fl / fused / 1e9, 1),
                      "unfused_ms": round(fc1 + fc2, 4), "fc1_ms": round(fc1, 4), "fc2_ms": round(fc2, 4)}))


if __name__ == "__main__":
    main()
