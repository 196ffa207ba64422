"""GEMM microbenchmark: every NT / TN shape of the ViT-S F1 step, kernel variants A/B'd in ONE
process (interleaved rounds, median), random operands.  Prints TFLOP/s per shape and variant.

  python scripts/gemm_bench.py [--variants 0,1] [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

M_T, M_W = 512 * 197, 448 * 197
D, HD = 384, 1536
# (name, epi, M, N, K)  -- NT: C[M,N] = A[M,K] B[N,K]^T; the engine's epilogues (data gradients of the LN
# inputs in bf16: Engine.DH_BF16)
NT = [("qkv_fwd", 0, M_T, 3 * D, D), ("proj_fwd", 2, M_T, D, D), ("fc1_fwd", 7, M_T, HD, D),
      ("fc2_fwd", 2, M_T, D, HD), ("fc1_fwd_weak", 6, M_W, HD, D), ("fc2_dgrad", 8, M_T, HD, D),
      ("fc1_dgrad", 0, M_T, D, HD), ("proj_dgrad", 0, M_T, D, D), ("qkv_dgrad", 0, M_T, D, 3 * D),
      ("qkv_fwd_weak", 0, M_W, 3 * D, D), ("proj_fwd_weak", 2, M_W, D, D), ("fc2_fwd_weak", 2, M_W, D, HD),
      ("patch_fwd", 5, 512 * 196, D, 768), ("patch_fwd_weak", 5, 448 * 196, D, 768),
      ("kv_fwd_last", 0, M_T, 2 * D, D), ("kv_fwd_last_weak", 0, M_W, 2 * D, D)]  # last block: K / V only
# (name, M, N1, N2)  -- TN: out[N1,N2] = sum_m A1[m,N1] A2[m,N2]
TN = [("fc2_wgrad", M_T, D, HD), ("fc1_wgrad", M_T, HD, D), ("proj_wgrad", M_T, D, D), ("qkv_wgrad", M_T, 3 * D, D)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--tn-variants", default="0,2")
    ap.add_argument("--tn-blocks", default="512", help="target workgroup counts (split-K sizing) to sweep; "
                    "'auto' = the library's sizing, 's<N>' = N splits")
    ap.add_argument("--m-train", type=int, default=0, help="token rows of the TN shapes (default 512 x 197)")
    ap.add_argument("--shard", type=int, default=1, help="F1 shapes at 1/N of the batch (a rank's share of the "
                    "global batch at N GPUs, strong scaling)")
    ap.add_argument("--s1", action="store_true", help="the Conformer-B/384 transformer-branch shapes of S1 "
                    "(D 768, hidden 3072, 120 images x 577 tokens)")
    args = ap.parse_args()
    global TN, NT
    if args.s1:
        m, d, hd = 120 * 577, 768, 3072
        NT = [("qkv_fwd", 0, m, 3 * d, d), ("proj_fwd", 2, m, d, d), ("fc1_fwd", 7, m, hd, d), ("fc2_fwd", 2, m, d, hd),
              ("fc2_dgrad", 8, m, hd, d), ("fc1_dgrad", 0, m, d, hd), ("proj_dgrad", 0, m, d, d),
              ("qkv_dgrad", 0, m, d, 3 * d), ("fc2_dgrad_dgelu", 3, m, hd, d), ("fc1_fwd_gelu", 1, m, hd, d),
              ("fc2_dgrad_plain", 0, m, hd, d)]
        TN = [("fc2_wgrad", m, d, hd), ("fc1_wgrad", m, hd, d), ("proj_wgrad", m, d, d), ("qkv_wgrad", m, 3 * d, d)]
    if args.shard > 1 and not args.s1:
        NT = [(n, e, M // args.shard, N, K) for n, e, M, N, K in NT]
        TN = [(n, M // args.shard, a, b) for n, M, a, b in TN]
    if args.m_train:
        TN = [(n, args.m_train, a, b) for n, _, a, b in TN]
    WX = max(max(n, k) for _, _, _, n, k in NT)  # widest operand / output row
    lib = _lib.load()
    lib.es_set_gemm_variant.restype = _lib.I
    lib.es_set_gemm_variant.argtypes = [_lib.I]
    lib.es_set_tn_variant.restype = _lib.I
    lib.es_set_tn_variant.argtypes = [_lib.I]
    tn_variants = [int(v) for v in args.tn_variants.split(",")]
    variants = [int(v) for v in args.variants.split(",")]
    dev = "cuda"
    torch.manual_seed(0)
    s = _lib.stream()
    Mp = (max(M for _, _, M, _, _ in NT) + 255) // 256 * 256
    A = torch.randn(Mp, max(WX, HD * 2), device=dev).bfloat16()
    Bw = (torch.randn(max(WX, HD * 2), max(WX, HD * 2), device=dev) * 0.05).bfloat16()
    bias = torch.randn(max(WX, HD * 2), device=dev)
    C = torch.empty(Mp, WX, device=dev)  # f32 [M, widest N]
    C2 = torch.empty(Mp, WX, device=dev, dtype=torch.bfloat16)
    aux = torch.randn(Mp, WX, device=dev)
    results = {}
    only = set(args.only.split(",")) if args.only else None
    for name, epi, M, N, K in NT:
        if only and name not in only:
            continue
        flops = 2.0 * M * N * K
        times = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                if N % {6: 256, 10: 128}.get(v, 128):
                    continue
                lib.es_set_gemm_variant(v)
                auxp = aux if epi in (2, 5) else (aux.bfloat16() if epi in (3, 8) else None)
                st = [ptr(A), K, ptr(Bw), K, ptr(bias) if epi not in (3, 4, 8) else None, ptr(C), N,
                      ptr(C2) if epi in (1, 7) else None, ptr(auxp) if auxp is not None else None, N, M, N, K, 196 if epi == 5 else 0, s]
                call("es_gemm_nt", epi, *st)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    call("es_gemm_nt", epi, *st)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.iters)
        row = {}
        for v in variants:
            if not times[v]:
                continue
            t = sorted(times[v])[len(times[v]) // 2]
            row[v] = {"ms": round(t, 4), "tflops": round(flops / t / 1e9, 1)}
        results[name] = row
        print(name, json.dumps(row), flush=True)
    ws = torch.empty(160 * max(n1 * n2 for _, _, n1, n2 in TN), device=dev)
    out = torch.empty(max(n1 * n2 for _, _, n1, n2 in TN), device=dev)
    for name, M, N1, N2 in TN:
        if only and name not in only:
            continue
        flops = 2.0 * M * N1 * N2
        tiles = (N1 // 128) * (N2 // 128)
        row = {}
        for tbs in args.tn_blocks.split(","):  # "768": ceil(768 / tiles) splits; "f768": floor
            if tbs == "auto":  # es_gemm_tn sizes the split-K for the kernel it picks
                splits = 0
            elif tbs.startswith("s"):
                splits = int(tbs[1:])
            else:
                tb = int(tbs.lstrip("f"))
                sp = tb // tiles if tbs.startswith("f") else -(-tb // tiles)
                splits = max(1, min((M + 31) // 32, sp))
            times = {v: [] for v in tn_variants}
            for _ in range(args.rounds):
                for v in tn_variants:
                    lib.es_set_tn_variant(v)
                    call("es_gemm_tn", ptr(A), N1, ptr(A), N2, M, N1, N2, splits, ptr(ws), ptr(out), 0, ptr(bias), s)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        call("es_gemm_tn", ptr(A), N1, ptr(A), N2, M, N1, N2, splits, ptr(ws), ptr(out), 0, ptr(bias),
                             s)
                    e1.record()
                    torch.cuda.synchronize()
                    times[v].append(e0.elapsed_time(e1) / args.iters)
            lib.es_set_tn_variant(-1)
            for v in tn_variants:
                t = sorted(times[v])[len(times[v]) // 2]
                row[f"tn{v}_b{tbs}"] = {"ms": round(t, 4), "tflops": round(flops / t / 1e9, 1), "splits": splits}
        results[name] = row
        print(name, json.dumps(row), flush=True)
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    json.dump(results, open(os.path.join(out_dir, "gemm_bench.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
