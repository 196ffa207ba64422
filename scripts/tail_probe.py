"""Probe: the 256 x 128 two-workgroup tile's last-round tail at the F1 fc2 / qkv / fc1 shapes.  Times each
shape at its M and at the M that fills whole rounds (512 resident workgroups), plus the remainder rows on
the 64 x 128 tile (variant 11): what splitting the launch would give in isolation.
  python scripts/tail_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

MT, MW = 512 * 197, 448 * 197
SH = [("fc2_fwd", 2, MT, 384, 1536), ("fc2_fwd_weak", 2, MW, 384, 1536), ("qkv_fwd_weak", 0, MW, 1152, 384),
      ("fc1_fwd", 7, MT, 1536, 384), ("proj_dgrad", 0, MT, 384, 384), ("fc2_dgrad", 8, MT, 1536, 384)]


def main():
    lib = _lib.load()
    s = _lib.stream()
    Mx = MT + 512
    A = torch.randn(Mx, 1536, device="cuda").bfloat16()
    B = (torch.randn(1536, 1536, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(1536, device="cuda")
    C = torch.empty(Mx, 1536, device="cuda")
    C2 = torch.empty(Mx, 1536, device="cuda", dtype=torch.bfloat16)
    aux = torch.randn(Mx, 1536, device="cuda")

    def t(epi, M, N, K, v=-1, it=20):
        old = lib.es_set_gemm_variant(v)
        auxp = aux if epi == 2 else (aux.bfloat16() if epi == 8 else None)
        args = [ptr(A), K, ptr(B), K, ptr(bias) if epi != 8 else None, ptr(C), N, ptr(C2) if epi == 7 else None,
                ptr(auxp) if auxp is not None else None, N, M, N, K, 0, s]
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
        lib.es_set_gemm_variant(old)
        return round(sorted(res)[2], 1)

    for name, epi, M, N, K in SH:
        ntn = N // 128
        rt = (M + 255) // 256
        full = (rt * ntn) // 512 * 512 // ntn  # row tiles that fill whole rounds
        M1 = full * 256
        print(name, json.dumps({"M": M, "wgs": rt * ntn, "us": t(epi, M, N, K), "M_full": M1, "wgs_full": full * ntn,
                                "us_full": t(epi, M1, N, K), "rem_rows": M - M1,
                                "rem_us_v11": t(epi, M - M1, N, K, 11) if M > M1 else 0}), flush=True)


if __name__ == "__main__":
    main()
