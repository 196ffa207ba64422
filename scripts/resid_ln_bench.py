"""es_gemm_nt_resid_ln (projection + residual + norm2 in one launch) vs es_gemm_nt(EPI_F32_RESID) +
es_layernorm_fwd at the F1 train / weak and N = 8 shard row counts: bit-identity and interleaved timings (µs).
  python scripts/resid_ln_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

D, EPS = 384, 1e-6


def main():
    _lib.load()
    s = _lib.stream()
    for name, M in (("f1_train", 512 * 197), ("f1_weak", 448 * 197), ("n2_train", 256 * 197), ("n2_weak", 224 * 197),
                    ("n4_train", 128 * 197), ("n4_weak", 112 * 197), ("shard_train", 64 * 197),
                    ("shard_weak", 56 * 197)):
        torch.manual_seed(0)
        A = torch.randn((M + 255) // 256 * 256, D, device="cuda").bfloat16()
        W = (torch.randn(D, D, device="cuda") * 0.05).bfloat16()
        bias = torch.randn(D, device="cuda") * 0.1
        xin = torch.randn(M, D, device="cuda")
        g, b = 1 + 0.1 * torch.randn(D, device="cuda"), 0.1 * torch.randn(D, device="cuda")
        outs = [(torch.empty(M, D, device="cuda"), torch.empty(M, D, dtype=torch.bfloat16, device="cuda"),
                 torch.empty(M, device="cuda"), torch.empty(M, device="cuda")) for _ in range(2)]

        def two(o):
            call("es_gemm_nt", 2, ptr(A), D, ptr(W), D, ptr(bias), ptr(o[0]), D, None, ptr(xin), D, M, D, D, 0, s)
            call("es_layernorm_fwd", ptr(o[0]), D, ptr(g), ptr(b), ptr(o[1]), D, ptr(o[2]), ptr(o[3]), M, D, EPS, s)

        def one(o):
            call("es_gemm_nt_resid_ln", ptr(A), D, ptr(W), D, ptr(bias), ptr(o[0]), D, ptr(xin), D, ptr(g), ptr(b),
                 ptr(o[1]), D, ptr(o[2]), ptr(o[3]), M, D, D, EPS, s)

        two(outs[0])
        one(outs[1])
        torch.cuda.synchronize()
        same = all(torch.equal(a, c) for a, c in zip(*outs))
        t = {"two": [], "one": []}
        it = 20
        for _ in range(5):
            for k, f in (("two", two), ("one", one)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(it):
                    f(outs[0])
                e1.record()
                torch.cuda.synchronize()
                t[k].append(e0.elapsed_time(e1) / it * 1e3)
        print(name, json.dumps({"bit_identical": same, **{k + "_us": round(sorted(v)[2], 1) for k, v in t.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
