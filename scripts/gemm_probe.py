"""Probe (shape from env N, K; EPIS, VARIANTS lists) what bounds a long-K NT GEMM (fc2 forward shape, M=100864 N=384 K=1536): the same launch with
A read from HBM vs an L2-resident aliased A (lda = 8: rows overlap), for several epilogues.

  python scripts/gemm_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402


EPIS = [(e, n) for e, n in ((4, "f32"), (0, "bf16"), (2, "f32_resid"), (7, "gelu_d"))
        if str(e) in os.environ.get("EPIS", "4,0,2").split(",")]


def main():
    lib = _lib.load()
    lib.es_set_gemm_variant.restype = _lib.I
    lib.es_set_gemm_variant.argtypes = [_lib.I]
    s = _lib.stream()
    M, N, K = 512 * 197, int(os.environ.get("N", 384)), int(os.environ.get("K", 1536))
    A = torch.randn(M, K, device="cuda").bfloat16()
    Bw = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    C = torch.empty(M, N, device="cuda")
    C2 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.randn(M, N, device="cuda")
    bias = torch.randn(N, device="cuda")
    for v in [int(x) for x in os.environ.get("VARIANTS", "1").split(",")]:
        lib.es_set_gemm_variant(v)
        for epi, name in EPIS:
            for lda, tag in ((K, "hbm"), (8, "l2")):
                args = [ptr(A), lda, ptr(Bw), K, ptr(bias) if epi != 4 else None, ptr(C), N, ptr(C2) if epi == 7 else None,
                        ptr(aux) if epi == 2 else None, N, M, N, K, 0, s]
                call("es_gemm_nt", epi, *args)
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        call("es_gemm_nt", epi, *args)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / 10)
                ts.sort()
                ms = ts[2]
                print(f"variant {v} epi {name:9s} A {tag}: {ms * 1e3:7.1f} us  {2 * M * N * K / ms / 1e9:6.1f} TF/s",
                      flush=True)


if __name__ == "__main__":
    main()
