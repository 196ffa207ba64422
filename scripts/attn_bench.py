"""Attention microbenchmark at the F1 train shape (512 images x 6 heads x 197 tokens; --s1: 120 x 12 x 577), forward
occupancy variants A/B'd in one process (interleaved rounds, median); backward (dQ + dK/dV).

  python scripts/attn_bench.py [--rounds 5] [--iters 10] [--save out.pt | --compare out.pt]
(--save / --compare: the outputs of one build against another's, bit for bit -- run the first under
ENDOSSL_LIB=<other build>)
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


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--s1", action="store_true", help="the S1 shape instead: 120 images x 12 heads x 577 tokens "
                    "(Conformer-B at 384^2, the long-sequence kernels)")
    ap.add_argument("--bwd", default="0,1,2,3,4", help="backward variants to time (es_set_attn_bwd_variant)")
    ap.add_argument("--no-fwd", action="store_true", help="skip the forward occupancy variants")
    ap.add_argument("--save", default=None, help="torch.save the outputs (forward o / lse, backward dqkv)")
    ap.add_argument("--compare", default=None, help="compare the outputs bit for bit with a --save file")
    args = ap.parse_args()
    bwd_vs = [int(v) for v in args.bwd.split(",")]
    lib = _lib.load()
    n, T, H = (120, 577, 12) if args.s1 else (512, 197, 6)
    D = 64 * H
    M = n * T
    torch.manual_seed(0)
    qkv = (torch.randn(M, 3 * D, device="cuda") * 0.5).bfloat16()
    o = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(n * H * T, device="cuda")
    delta = torch.empty(n * H * T, device="cuda")
    do = torch.randn(M, D, device="cuda").bfloat16()
    dqkv = torch.empty(M, 3 * D, device="cuda", dtype=torch.bfloat16)
    s = _lib.stream()
    fwd = lambda: call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 0.125, s)  # noqa: E731
    bwd = lambda: call("es_attn_bwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), ptr(delta), ptr(do), D, ptr(dqkv),  # noqa
                       3 * D, n, T, H, 0.125, s)
    res = {"fwd_occ2": [], "fwd_occ3": [], "fwd_occ7": [], "bwd_plain": [], "bwd_pipe": [], "bwd_dkv2": [],
           "bwd_dq2_dkv2": [], "bwd_fused": []}
    outs = {}
    for _ in range(args.rounds):
        for occ in (() if args.no_fwd else (2, 3, 7)):  # 7: seven waves per workgroup (T = 197)
            lib.es_set_attn_variant(occ)
            res[f"fwd_occ{occ}"].append(timed(fwd, args.iters))
            outs[f"fwd_occ{occ}"] = (o.clone(), lse.clone())
        lib.es_set_attn_variant(2)
        fwd()
        for v, name in ((0, "bwd_plain"), (1, "bwd_pipe"), (2, "bwd_dkv2"), (3, "bwd_dq2_dkv2"), (4, "bwd_fused")):
            if v not in bwd_vs:
                continue
            lib.es_set_attn_bwd_variant(v)
            res[name].append(timed(bwd, args.iters))
            outs[name] = dqkv.clone()
    lib.es_set_attn_bwd_variant(4)
    if not args.no_fwd:
        print("fwd occ7 == occ2 (bit-exact):",
              all(torch.equal(x, y) for x, y in zip(outs["fwd_occ7"], outs["fwd_occ2"])), flush=True)
    if "bwd_plain" in outs:
        print("bwd == plain (bit-exact):", {k: torch.equal(v, outs["bwd_plain"]) for k, v in outs.items()
                                            if k.startswith("bwd_")}, flush=True)
    if args.save:
        torch.save({k: (tuple(x.cpu() for x in v) if isinstance(v, tuple) else v.cpu()) for k, v in outs.items()},
                   args.save)
    if args.compare:
        ref = torch.load(args.compare, weights_only=True)
        same = {}
        for k, v in outs.items():
            if k in ref:
                a = v if isinstance(v, tuple) else (v,)
                b = ref[k] if isinstance(ref[k], tuple) else (ref[k],)
                same[k] = all(torch.equal(x.cpu(), y) for x, y in zip(a, b))
        print("bit-identical to", args.compare, same, flush=True)
    flops_f = 4.0 * n * H * T * T * 64
    out = {}
    for k, v in res.items():
        if not v:
            continue
        t = sorted(v)[len(v) // 2]
        fl = flops_f if k.startswith("fwd") else 2.5 * flops_f
        out[k] = {"ms": round(t, 4), "tflops": round(fl / t / 1e9, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
