"""The per-block bf16-contract oracle (oracle/ref.py block_fwd_bf16 / block_bwd_bf16) that the
teacher-forced GPU test (tests/test_gpu_blocks.py) holds the production kernels to, checked on the CPU:

  * forward: the embedding + 12-step block chain + head equals the oracle's whole-model bf16-contract
    forward (vit_forward(bf16=True), itself the fp32 arithmetic pinned to the reference's fixtures by
    test_oracle_golden.py) -- the same rounding points, op for op;
  * reverse pass: with the rounding points switched off, block_bwd_bf16 equals torch.autograd through
    block_fwd_bf16 in float64 (every parameter gradient and dx), and so is the exact derivative of
    code/models/conformer.py:53-72's Block; with them on, it stays within the bf16 envelope of it.
"""
import pytest
import torch

from oracle import ref


@pytest.fixture
def tiny():
    cfg = ref.Cfg(img_size=64, patch=16, dim=128, depth=2, heads=2, num_classes=23)
    p = ref.random_params(cfg, seed=4, head_std=0.5)
    return cfg, p


def test_block_chain_equals_whole_model_bf16_forward(tiny):
    cfg, p = tiny
    x = torch.randn(3, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    t = ref.embed_fwd_bf16(p, x, cfg)
    for i in range(cfg.depth):
        t, _ = ref.block_fwd_bf16(p, i, t, 3, cfg)
    logits = ref.head_fwd(p, t.view(3, cfg.T, cfg.dim)[:, 0], cfg)
    want = ref.vit_forward(p, x, cfg, bf16=True)
    # same rounding points; only the LayerNorm statistics' fp32 evaluation order differs
    torch.testing.assert_close(logits, want, rtol=1e-4, atol=1e-4 * want.abs().max().item())


def test_block_reverse_pass_is_autograd_without_rounding(tiny):
    cfg, p = tiny
    n = 2
    p64 = {k: v.double().requires_grad_(True) for k, v in p.items()}
    g = torch.Generator().manual_seed(2)
    x = torch.randn(n * cfg.T, cfg.dim, generator=g, dtype=torch.float64, requires_grad=True)
    dy = torch.randn(n * cfg.T, cfg.dim, generator=g, dtype=torch.float64)
    old = ref.ROUND
    ref.ROUND = False
    try:
        out, cache = ref.block_fwd_bf16(p64, 1, x, n, cfg)
        out.backward(dy)
        dx, grads = ref.block_bwd_bf16({k: v.detach() for k, v in p64.items()}, 1,
                                       {k: v.detach() for k, v in cache.items()}, dy, n, cfg)
    finally:
        ref.ROUND = old
    torch.testing.assert_close(dx, x.grad, rtol=1e-10, atol=1e-12)
    assert len(grads) == 12
    for k, gk in grads.items():
        torch.testing.assert_close(gk, p64[k].grad, rtol=1e-10, atol=1e-12 * max(1.0, p64[k].grad.abs().max().item()))


def test_block_reverse_pass_rounding_stays_in_bf16_envelope(tiny):
    cfg, p = tiny
    n = 2
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n * cfg.T, cfg.dim, generator=g)
    dy = torch.randn(n * cfg.T, cfg.dim, generator=g)
    out, cache = ref.block_fwd_bf16(p, 0, x, n, cfg)
    dx, grads = ref.block_bwd_bf16(p, 0, cache, dy, n, cfg)
    old = ref.ROUND
    ref.ROUND = False
    try:
        out0, cache0 = ref.block_fwd_bf16(p, 0, x, n, cfg)
        dx0, grads0 = ref.block_bwd_bf16(p, 0, cache0, dy, n, cfg)
    finally:
        ref.ROUND = old
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert 0 < rel(out - x, out0 - x) < 2e-2
    assert 0 < rel(dx - dy, dx0 - dy) < 3e-2
    for k in grads:
        assert rel(grads[k], grads0[k]) < 3e-2, k
