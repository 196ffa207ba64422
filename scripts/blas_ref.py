"""Calibration only: torch bf16 matmul (hipBLASLt) on the ViT-S F1 GEMM shapes, to see what the vendor
library reaches on these skinny M-huge shapes.  Not used by the framework."""
import json
import torch

M_T, M_W, D, HD = 512 * 197, 448 * 197, 384, 1536
shapes = [("qkv_fwd", M_T, 3 * D, D), ("proj_fwd", M_T, D, D), ("fc1_fwd", M_T, HD, D), ("fc2_fwd", M_T, D, HD),
          ("fc1_dgrad", M_T, D, HD), ("qkv_dgrad", M_T, D, 3 * D), ("sq4096", 4096, 4096, 4096)]
out = {}
for name, M, N, K in shapes:
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(N, K, device="cuda").bfloat16()
    for _ in range(3):
        c = a @ b.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        c = a @ b.t()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10
    out[name] = {"ms": round(t, 4), "tflops": round(2.0 * M * N * K / t / 1e9, 1)}
    print(name, out[name], flush=True)
    # wgrad form: [N, M] x [M, K]
    if name in ("fc2_fwd", "fc1_fwd"):
        g = torch.randn(M, N, device="cuda").bfloat16()
        for _ in range(3):
            w = g.t() @ a
        e0.record()
        for _ in range(10):
            w = g.t() @ a
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 10
        print(name + "_wgrad", {"ms": round(t, 4), "tflops": round(2.0 * M * N * K / t / 1e9, 1)}, flush=True)
