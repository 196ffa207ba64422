"""Probe: would a 2-way split-K help the long-K N = 384 GEMMs of the N = 8 shard?  Times each shape and the
same shape with M doubled and K halved (twice the workgroups, half the K chain each: the split kernel's main
loop without its fix-up).  python scripts/splitk_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

M8, MW8 = 64 * 197, 56 * 197
SH = [("fc2_fwd", 2, M8, 384, 1536), ("fc2_fwd_weak", 2, MW8, 384, 1536), ("fc1_dgrad", 0, M8, 384, 1536),
      ("qkv_dgrad", 0, M8, 384, 1152), ("proj_fwd", 2, M8, 384, 384), ("proj_dgrad", 0, M8, 384, 384)]


def main():
    _lib.load()
    s = _lib.stream()
    Mx = 4 * M8 + 256
    A = torch.randn(Mx, 1536, device="cuda").bfloat16()
    B = (torch.randn(1536, 1536, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(1536, device="cuda")
    C = torch.empty(Mx, 1536, device="cuda")
    aux = torch.randn(Mx, 1536, device="cuda")

    def t(epi, M, N, K, it=50):
        args = [ptr(A), K, ptr(B), K, ptr(bias), ptr(C), N, None, ptr(aux) if epi == 2 else None, N, M, N, K, 0, s]
        for _ in range(3):
            call("es_gemm_nt", epi, *args)
        res = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(it):
                call("es_gemm_nt", epi, *args)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / it * 1e3)
        return round(sorted(res)[2], 1)

    lib = _lib.load()
    for name, epi, M, N, K in SH:
        row = {"us": t(epi, M, N, K)}
        for v in (0, 2, 10):
            old = lib.es_set_gemm_variant(v)
            row[f"v{v}"] = t(epi, M, N, K)
            row[f"v{v}_2M_halfK"] = t(epi, 2 * M, N, K // 2)
            if K % 256 == 0 and v == 10:
                row[f"v{v}_4M_quarterK"] = t(epi, 4 * M, N, K // 4)
            lib.es_set_gemm_variant(old)
        print(name, json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
