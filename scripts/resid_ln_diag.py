"""Diagnostic for es_gemm_nt_resid_ln vs the two-launch form: where outputs differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

D, EPS = 384, 1e-6
s = _lib.stream()
for M in (777, 64):
    torch.manual_seed(M)
    A = torch.randn((M + 255) // 256 * 256, D, device="cuda").bfloat16()
    W = (torch.randn(D, D, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(D, device="cuda") * 0.1
    xin = torch.randn(M, D, device="cuda")
    g, b = 1 + 0.1 * torch.randn(D, device="cuda"), 0.1 * torch.randn(D, device="cuda")
    nan = float("nan")
    o0 = [torch.full((M, D), nan, device="cuda"), torch.full((M, D), nan, dtype=torch.bfloat16, device="cuda"),
          torch.full((M,), nan, device="cuda"), torch.full((M,), nan, device="cuda")]
    o1 = [t.clone() for t in o0]
    call("es_gemm_nt", 2, ptr(A), D, ptr(W), D, ptr(bias), ptr(o0[0]), D, None, ptr(xin), D, M, D, D, 0, s)
    call("es_layernorm_fwd", ptr(o0[0]), D, ptr(g), ptr(b), ptr(o0[1]), D, ptr(o0[2]), ptr(o0[3]), M, D, EPS, s)
    call("es_gemm_nt_resid_ln", ptr(A), D, ptr(W), D, ptr(bias), ptr(o1[0]), D, ptr(xin), D, ptr(g), ptr(b),
         ptr(o1[1]), D, ptr(o1[2]), ptr(o1[3]), M, D, D, EPS, s)
    torch.cuda.synchronize()
    ref = A[:M].float() @ W.float().t() + bias + xin
    for nm, a, c in zip(("x", "h", "mean", "rstd"), o0, o1):
        a, c = a.float(), c.float()
        bad = ~((a == c) | (torch.isnan(a) & torch.isnan(c)))
        print(M, nm, "mismatch", int(bad.sum()), "nan_ref", int(torch.isnan(a).sum()), "nan_new", int(torch.isnan(c).sum()),
              "maxdiff", float((a - c).abs().nan_to_num(0).max()))
        if nm == "x":
            print("   ref-vs-torch", float((a - ref).abs().max()), "new-vs-torch", float((c - ref).abs().nan_to_num(1e9).max()))
        if int(bad.sum()):
            idx = bad.nonzero()[:6].tolist()
            print("   first", idx, [(float(a[tuple(i)]), float(c[tuple(i)])) for i in idx])
            if a.dim() == 2:
                rows = bad.any(1).nonzero().flatten()
                cols = bad.any(0).nonzero().flatten()
                print("   rows", rows[:20].tolist(), len(rows), "cols", cols[:20].tolist(), len(cols))
            else:
                rows = bad.nonzero().flatten()
                print("   rows", rows[:30].tolist(), "parity counts", int((rows % 2 == 0).sum()), int((rows % 2 == 1).sum()))
