"""LayerNorm forward microbenchmark at the F1 shape (M = 512 x 197 tokens, D = 384): es_set_ln_fwd_grid values
A/B'd in one process (interleaved rounds, median ms), outputs checked bit-identical to the one-shot kernel.
  python scripts/ln_bench.py [--grids 0,1024,2048] [--rounds 5] [--iters 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="0,512,1024,2048,4096")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=512 * 197)
    args = ap.parse_args()
    lib = _lib.load()
    M, D = args.m, 384
    torch.manual_seed(0)
    x = torch.randn(M, D, device="cuda") * 3 + 0.5
    g, b = torch.randn(D, device="cuda"), torch.randn(D, device="cuda")
    y = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    mu, rs = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    s = _lib.stream()
    grids = [int(v) for v in args.grids.split(",")]
    times, outs = {v: [] for v in grids}, {}
    for _ in range(args.rounds):
        for v in grids:
            lib.es_set_ln_fwd_grid(v)
            f = lambda: call("es_layernorm_fwd", ptr(x), D, ptr(g), ptr(b), ptr(y), D, ptr(mu), ptr(rs), M, D, 1e-6, s)  # noqa
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters)
            outs[v] = (y.clone(), mu.clone(), rs.clone())
    lib.es_set_ln_fwd_grid(0)
    ref = outs[grids[0]]
    byts = M * D * 4 + M * D * 2 + 8 * M
    res = {v: {"ms": round(sorted(t)[len(t) // 2], 4), "TB/s": round(byts / sorted(t)[len(t) // 2] / 1e9, 2),
               "bit_identical": all(torch.equal(a, c) for a, c in zip(outs[v], ref))} for v, t in times.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
