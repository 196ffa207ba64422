"""Overlapped gradient all-reduce on the GPU path: two ranks share cuda:0 (gloo over HIP tensors --
the box has one GPU, and RCCL refuses two ranks on one device), each runs the native ViT reverse
pass on its own shard with Engine.backward's per-block hook driving dist.GradBuckets (all-reduces
issued from a comm stream that waits on the engine's HIP events, beside the remaining backward
kernels).  Bar: the transformer blocks' gradients bit-identical to the same backward followed by
one whole-buffer all-reduce, on every rank, with one bucket per block handed over (the rest within
fp32 summation order, and only on tensors that already differ between two local backward passes:
the head reduction uses fp32 atomics)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
    from endossl import dist
    from endossl.vit import NativeViT, ViTConfig
    dist.init_from_env(backend="gloo")
    try:
        cfg = ViTConfig(img_size=64, dim=128, depth=3, heads=2, num_classes=23)
        m = NativeViT(cfg, seed=3).to("cuda")
        eng = m.engine()
        eng.pack(m.flat, m.version)
        g = torch.Generator(device="cuda").manual_seed(10 + rank)
        x = torch.randn(64, 3, 64, 64, device="cuda", generator=g)
        dl = torch.randn(64, 23, device="cuda", generator=g) * 1e-2
        eng.forward(m.flat, [x], train=True)
        # local reverse pass twice, no collective: which entries are run-to-run deterministic
        ga, gc = torch.zeros_like(m.flat), torch.zeros_like(m.flat)
        eng.backward(m.flat, ga, dlogits=dl)
        eng.backward(m.flat, gc, dlogits=dl)
        torch.cuda.synchronize()
        nondet = [name for name, _ in eng.layout if not torch.equal(eng.view(ga, name), eng.view(gc, name))]
        g_serial = torch.zeros_like(m.flat)
        eng.backward(m.flat, g_serial, dlogits=dl)
        s1 = dist.allreduce_sum_(g_serial)
        g_b = torch.zeros_like(m.flat)
        gb = dist.GradBuckets(g_b)
        eng.backward(m.flat, g_b, dlogits=dl, grad_ready=gb.ready)
        ranges = list(gb.ranges)
        s2 = gb.finish()
        torch.cuda.synchronize()
        # block ranges (split-K GEMM + per-workgroup partial reductions: deterministic) bit for bit;
        # the whole buffer within fp32 summation order (the head / embedding reductions use atomics)
        blocks_same = all(torch.equal(g_serial[lo:hi], g_b[lo:hi]) for lo, hi in ranges)
        close = torch.allclose(g_serial, g_b, rtol=1e-5, atol=1e-6)
        differ = [name for name, _ in eng.layout if not torch.equal(eng.view(g_serial, name), eng.view(g_b, name))]
        diff = f"{float((g_serial - g_b).abs().max())}; differing {differ}; local run-to-run nondeterministic {nondet}"
        q.put((rank, blocks_same and close and set(differ) <= set(nondet), diff, s1, s2, len(ranges),
               float(g_b[ranges[-1][0]:ranges[0][1]].abs().sum())))
        dist.barrier()
    finally:
        torch.distributed.destroy_process_group()


def test_two_rank_overlapped_allreduce_bit_identical():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sums = set()
    for rank, same, diff, s1, s2, handed, gsum in res:
        assert same, f"rank {rank}: overlapped all-reduce differs by {diff}"
        assert s1 == s2 == 0.5
        assert handed == 3
        sums.add(gsum)
    assert len(sums) == 1  # both ranks hold the same summed block gradients
