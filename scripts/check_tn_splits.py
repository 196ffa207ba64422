"""es_gemm_tn at the S1 / F1 weight-gradient shapes: the split counts Engine.TN_SHARE / CONF_TN_SHARE pick vs
the library's automatic sizing vs a torch fp32 reference (max relative difference printed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

torch.manual_seed(0)
lib = _lib.load()
for M, N1, N2, sp in [(69240, 3072, 768, 4), (69240, 768, 3072, 4), (69240, 768, 768, 16), (100864, 1536, 384, 16),
                      (50432, 1152, 384, 21), (25216, 384, 384, 64)]:
    Mp = (M + 255) // 256 * 256
    dy = torch.zeros(Mp, N1, device="cuda", dtype=torch.bfloat16)
    x = torch.zeros(Mp, N2, device="cuda", dtype=torch.bfloat16)
    dy[:M] = torch.randn(M, N1, device="cuda").bfloat16()
    x[:M] = torch.randn(M, N2, device="cuda").bfloat16()
    ref = dy[:M].float().t() @ x[:M].float()
    outs = []
    for s in (0, sp):
        old = lib.es_set_tn_variant(7)
        ws = torch.empty(lib.es_gemm_tn_workspace(N1, N2, s), device="cuda")
        out = torch.empty(N1, N2, device="cuda")
        bias = torch.empty(N1, device="cuda")
        call("es_gemm_tn", ptr(dy), N1, ptr(x), N2, M, N1, N2, s, ptr(ws), ptr(out), 0, ptr(bias), _lib.stream())
        lib.es_set_tn_variant(old)
        torch.cuda.synchronize()
        outs.append(out)
    sc = ref.abs().max().item()
    print(M, N1, N2, sp, "auto vs ref %.2e" % ((outs[0] - ref).abs().max().item() / sc),
          "split vs ref %.2e" % ((outs[1] - ref).abs().max().item() / sc),
          "split vs auto %.2e" % ((outs[1] - outs[0]).abs().max().item() / sc), flush=True)
