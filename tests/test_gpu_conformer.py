"""Conformer / SemiFormer on the MI355X.

Kernels (conv.hip, es_ce_weighted_fwd_bwd) against plain torch fp64 CPU restatements of the same ops
(autograd for the gradients): fp32 tolerances.  The native Conformer against the oracle
(oracle/conformer_ref.py, pinned bit-exact to the reference's SemiFormer.train_one fixture): forward
logits within 1e-3 * scale of the bf16-contract emulation (the transformer blocks round their GEMM
operands to bf16; with fp32 convs) or within twice the contract's envelope of the fp32 reference
(bf16 convs, csrc/conv_bf16.hip, vs fp64 of rounded operands above); the SemiFormer trainer against the reference fixture over
two steps within the bf16 envelope, pseudo-labels / masks bit-exact on decidable rows, parameters
within 2 * lr * steps.
"""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402
from oracle import conformer_ref as cr  # noqa: E402

DEV = "cuda"


def S():
    return _lib.stream()


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    _lib.load()


_KEEP = []


@pytest.fixture(autouse=True)
def _keep_alive():
    """Device copies made inline in a call's argument list must outlive the launch: a temporary
    freed right after ptr() can hand its block to the next argument's copy (aliased operands)."""
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def dv(t, dtype=torch.float32):
    """A device copy kept alive until the end of the test."""
    t = t.to(dtype).to(DEV).contiguous()
    _KEEP.append(t)
    return t


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def _close(a, b, rtol=1e-4, atol=1e-4):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    sc = max(1.0, b.abs().max().item())
    err = (a - b).abs().max().item()
    assert err <= atol * sc, (err, sc)


# ------------------------------------------------------------------------------------ conv
@pytest.mark.parametrize("N,Cin,H,Cout,k,s,p", [(3, 5, 11, 7, 3, 2, 1), (2, 64, 16, 16, 1, 1, 0),
                                                (2, 16, 16, 16, 3, 1, 1), (2, 32, 12, 128, 1, 2, 0),
                                                (2, 64, 16, 96, 4, 4, 0), (1, 40, 9, 33, 3, 1, 1),
                                                (2, 3, 13, 20, 7, 2, 3), (2, 8, 10, 12, 2, 3, 0),
                                                (2, 16, 8, 64, 1, 1, 0), (2, 8, 10, 40, 2, 1, 0)])
def test_conv2d_fwd_bwd(N, Cin, H, Cout, k, s, p):
    torch.manual_seed(N * 100 + Cin + Cout)
    x = torch.randn(N, Cin, H, H, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, dtype=torch.float64) * 0.2
    b = torch.randn(Cout, dtype=torch.float64)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = F.conv2d(xr, wr, br, stride=s, padding=p)
    Ho = y.shape[2]
    xd, wd, bd = _nhwc(x).float().to(DEV), w.float().to(DEV), b.float().to(DEV)
    yd = torch.empty(N, Ho, Ho, Cout, device=DEV)
    call("es_conv2d_fwd", ptr(xd), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(wd), ptr(bd), Cout, k, k, s, p,
         ptr(yd), Ho * Ho * Cout, Ho * Cout, Cout, 0, S())
    _close(_nchw(yd.cpu()), y)
    dy = torch.randn_like(y)
    y.backward(dy)
    dyd = _nhwc(dy).float().to(DEV)
    dxd = torch.empty(N, H, H, Cin, device=DEV)
    call("es_conv2d_bwd_data", ptr(dyd), Ho * Ho * Cout, Ho * Cout, Cout, ptr(wd), N, H, H, Cin, Cout, k, k, s, p,
         ptr(dxd), H * H * Cin, H * Cin, Cin, 1, 0, S())
    _close(_nchw(dxd.cpu()), xr.grad)
    for splits in (1, 3, 40):
        ws = torch.empty(_lib.load().es_conv2d_bwd_weight_workspace(Cout, Cin, k, k, splits), device=DEV)
        dwd = torch.empty_like(wd)
        call("es_conv2d_bwd_weight", ptr(xd), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(dyd), Ho * Ho * Cout,
             Ho * Cout, Cout, Cout, k, k, s, p, splits, ptr(ws), ptr(dwd), 0, S())
        _close(dwd.cpu(), wr.grad)
    M = N * Ho * Ho
    wsb = torch.empty(_lib.load().es_chan_workspace(M, Cout), device=DEV)
    dbd = torch.full((Cout,), 3.0, device=DEV)
    call("es_chan_sum", ptr(dyd), M, Cout, M * Cout, Cout, M, ptr(wsb), ptr(dbd), 1, S())
    _close(dbd.cpu() - 3.0, br.grad)


@pytest.mark.parametrize("N,H", [(2, 40), (1, 150), (2, 224)])
def test_stem_conv_kernels(N, H):
    """The specialised 3 -> 64 channel 7x7 / 2 / 3 stem kernels (es_set_stem_kernels(1), the default)
    on NHWC fp32 images: forward bit-identical to the generic implicit-GEMM kernel (same (ky, kx, ci)
    fmaf order), both passes within fp32 tolerance of fp64 torch, the weight gradient also at a
    caller-sized slab count below the kernel's grid, with accumulate; partial 64-pixel row segments
    (Wo = 20, 75, 112)."""
    lib = _lib.load()
    torch.manual_seed(N + H)
    Cin, Cout, k, s, p = 3, 64, 7, 2, 3
    x = torch.randn(N, Cin, H, H, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, dtype=torch.float64) * 0.2
    b = torch.randn(Cout, dtype=torch.float64)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = F.conv2d(xr, wr, b, stride=s, padding=p)
    Ho = y.shape[2]
    xd, wd, bd = _nhwc(x).float().to(DEV), w.float().to(DEV), b.float().to(DEV)
    args = (ptr(xd), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(wd), ptr(bd), Cout, k, k, s, p)
    outs = {}
    for stem in (1, 0):
        old = lib.es_set_stem_kernels(stem)
        try:
            yd = torch.empty(N, Ho, Ho, Cout, device=DEV)
            call("es_conv2d_fwd", *args, ptr(yd), Ho * Ho * Cout, Ho * Cout, Cout, 0, S())
            torch.cuda.synchronize()
            outs[stem] = yd
        finally:
            lib.es_set_stem_kernels(old)
    assert torch.equal(outs[1], outs[0])
    _close(_nchw(outs[1].cpu()), y)
    dy = torch.randn_like(y)
    y.backward(dy)
    dyd = _nhwc(dy).float().to(DEV)
    for splits in (683, 7):
        ws = torch.empty(lib.es_conv2d_bwd_weight_workspace(Cout, Cin, k, k, splits), device=DEV)
        dwd = torch.full_like(wd, 0.5)
        call("es_conv2d_bwd_weight", ptr(xd), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(dyd), Ho * Ho * Cout,
             Ho * Cout, Cout, Cout, k, k, s, p, splits, ptr(ws), ptr(dwd), 1, S())
        _close(dwd.cpu() - 0.5, wr.grad)


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


@pytest.mark.parametrize("N,Cin,H,Cout,k,s,p", [(2, 64, 16, 64, 1, 1, 0), (2, 32, 13, 96, 3, 1, 1),
                                                (3, 64, 15, 128, 3, 2, 1), (2, 128, 12, 256, 1, 2, 0),
                                                (2, 64, 16, 384, 4, 4, 0), (1, 96, 9, 32, 3, 1, 1),
                                                (2, 256, 8, 64, 1, 1, 0)])
def test_conv2d_bf16_fwd_bwd(N, Cin, H, Cout, k, s, p):
    """csrc/conv_bf16.hip against fp64 convs of the bf16-rounded operands (the kernels' contract:
    operands rounded to bf16, fp32 accumulation): forward, data gradient, weight gradient (pixel
    splits 1, 3 and automatic), accumulate mode."""
    lib = _lib.load()
    assert lib.es_conv2d_bf16_eligible(Cin, Cout, k, k) == 1
    torch.manual_seed(N * 100 + Cin + Cout + k)
    x = torch.randn(N, Cin, H, H, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, dtype=torch.float64) * 0.2
    b = torch.randn(Cout, dtype=torch.float64)
    xr, wr = _bf(x).requires_grad_(True), _bf(w).requires_grad_(True)
    y = F.conv2d(xr, wr, b, stride=s, padding=p)
    Ho = y.shape[2]
    xd, wd, bd = _nhwc(x).float().to(DEV), w.float().to(DEV), b.float().to(DEV)
    n = Cout * Cin * k * k
    wp, wt = torch.empty(n, dtype=torch.bfloat16, device=DEV), torch.empty(n, dtype=torch.bfloat16, device=DEV)
    call("es_conv2d_pack_bf16", ptr(wd), Cout, Cin, k, k, ptr(wp), ptr(wt), S())
    torch.cuda.synchronize()
    assert torch.equal(wp.view(Cout, k * k, Cin).cpu(), w.float().bfloat16().view(Cout, Cin, k * k).transpose(1, 2))
    yd = torch.full((N, Ho, Ho, Cout), 0.5, device=DEV)
    call("es_conv2d_fwd_bf16", ptr(xd), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(wp), ptr(bd), Cout, k, k, s,
         p, ptr(yd), Ho * Ho * Cout, Ho * Cout, Cout, 1, S())
    _close(_nchw(yd.cpu()) - 0.5, y, atol=2e-5)
    dy = torch.randn_like(y)
    y.backward(_bf(dy))
    dyd = _nhwc(dy).float().to(DEV)
    dxd = torch.empty(N, H, H, Cin, device=DEV)
    call("es_conv2d_bwd_data_bf16", ptr(dyd), Ho * Ho * Cout, Ho * Cout, Cout, ptr(wt), N, H, H, Cin, Cout, k, k, s,
         p, ptr(dxd), H * H * Cin, H * Cin, Cin, 1, 0, S())
    _close(_nchw(dxd.cpu()), xr.grad, atol=2e-5)
    M = N * Ho * Ho
    for splits in (1, 3, 0):
        ws = torch.empty(lib.es_conv2d_bwd_weight_bf16_workspace(M, Cout, Cin, k, k, splits), device=DEV)
        dwd = torch.full_like(wd, 2.0)
        call("es_conv2d_bwd_weight_bf16", ptr(xd), N, H, H, Cin, H * H * Cin, H * Cin, Cin, 1, ptr(dyd),
             Ho * Ho * Cout, Ho * Cout, Cout, Cout, k, k, s, p, splits, ptr(ws), ptr(dwd), 1, S())
        _close(dwd.cpu() - 2.0, wr.grad, atol=2e-5)


@pytest.mark.parametrize("N,Cin,H,Cout,k,s,p", [(3, 64, 15, 64, 3, 1, 1), (2, 32, 20, 128, 1, 2, 0),
                                                (2, 64, 9, 256, 3, 1, 1), (5, 32, 45, 64, 1, 1, 0)])
def test_conv_bf16_fused_bn_statistics(N, Cin, H, Cout, k, s, p):
    """es_conv2d_fwd_bf16_bnstats (per-128-pixel-block sum / centred M2 in the conv epilogue) +
    es_bn2d_fwd_partials (Chan combination) give es_bn2d_fwd's statistics of the same conv output:
    the same y (bit-identical conv), mean / rstd / running stats within fp32 summation order, the
    normalised output too; pixel counts that are not multiples of 128 (a partial last block), and
    10,125 pixels = 80 blocks (the two-level combine with a partial last group)."""
    lib = _lib.load()
    torch.manual_seed(N + Cin + Cout)
    x = _nhwc(torch.randn(N, Cin, H, H)).to(DEV)
    w = (torch.randn(Cout, Cin, k, k) * 0.2).to(DEV)
    b = torch.randn(Cout).to(DEV) * 3.0  # a bias shifts the mean: the centring must follow it
    Ho = (H + 2 * p - k) // s + 1
    M = N * Ho * Ho
    wp = torch.empty(Cout * Cin * k * k, dtype=torch.bfloat16, device=DEV)
    call("es_conv2d_pack_bf16", ptr(w), Cout, Cin, k, k, ptr(wp), None, S())
    y1, y2 = torch.empty(M, Cout, device=DEV), torch.empty(M, Cout, device=DEV)
    geo = (H * H * Cin, H * Cin, Cin, 1)
    call("es_conv2d_fwd_bf16", ptr(x), N, H, H, Cin, *geo, ptr(wp), ptr(b), Cout, k, k, s, p, ptr(y1),
         Ho * Ho * Cout, Ho * Cout, Cout, 0, S())
    part = torch.empty(lib.es_conv2d_bnstats_size(M, Cout), device=DEV)
    call("es_conv2d_fwd_bf16_bnstats", ptr(x), N, H, H, Cin, *geo, ptr(wp), ptr(b), Cout, k, k, s, p, ptr(y2),
         Ho * Ho * Cout, Ho * Cout, Cout, ptr(part), S())
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    gam, bet = dv(torch.rand(Cout) + 0.5), dv(torch.randn(Cout))
    rm0, rv0 = torch.randn(Cout), torch.rand(Cout) + 0.5  # the same running stats entering both paths
    outs = []
    for fused in (False, True):
        rm, rvv, nbt = dv(rm0.clone()), dv(rv0.clone()), torch.zeros((), dtype=torch.int64, device=DEV)
        yo, mean, rstd = torch.empty_like(y1), torch.empty(Cout, device=DEV), torch.empty(Cout, device=DEV)
        if fused:
            call("es_bn2d_fwd_partials", ptr(y2), M, Cout, ptr(part), ptr(gam), ptr(bet), ptr(rm), ptr(rvv), ptr(nbt),
                 0.1, 1e-6, None, 1, ptr(yo), ptr(mean), ptr(rstd), S())
        else:
            ws = torch.empty(lib.es_chan_workspace(M, Cout), device=DEV)
            call("es_bn2d_fwd", ptr(y1), M, Cout, ptr(gam), ptr(bet), ptr(rm), ptr(rvv), ptr(nbt), 0.1, 1e-6, 1, None,
                 1, ptr(yo), ptr(mean), ptr(rstd), ptr(ws), S())
        torch.cuda.synchronize()
        outs.append((yo.cpu(), mean.cpu(), rstd.cpu(), rm.cpu(), rvv.cpu(), int(nbt.item())))
    ref = y1.double().cpu()
    mu, var = ref.mean(0), ref.var(0, unbiased=False)
    for i, (a, c) in enumerate(zip(outs[0], outs[1])):
        if isinstance(a, int):
            assert a == c == 1
        else:
            _close(c, a, atol=2e-5)
    _close(outs[1][1], mu, atol=1e-5)
    _close(outs[1][2], 1.0 / (var + 1e-6).sqrt(), atol=1e-4)


def test_conv2d_bf16_token_rows():
    """bf16 convs over token-row views: a 4x4/4 patch conv written into rows 1.. of [N, T, D]
    (trans_patch_conv), and a 1x1 conv reading them back with its data gradient written into token
    rows (FCUUp conv_project), row 0 untouched."""
    torch.manual_seed(5)
    N, C, H, D, k = 2, 64, 24, 128, 4
    g = H // k
    T = g * g + 1
    x = torch.randn(N, C, H, H)
    w = torch.randn(D, C, k, k) * 0.1
    wp = torch.empty(D * C * k * k, dtype=torch.bfloat16, device=DEV)
    call("es_conv2d_pack_bf16", ptr(dv(w)), D, C, k, k, ptr(wp), None, S())
    tok = torch.full((N * T, D), 9.0, device=DEV)
    call("es_conv2d_fwd_bf16", ptr(dv(_nhwc(x))), N, H, H, C, H * H * C, H * C, C, 1, ptr(wp), None, D, k, k, k, 0,
         ptr(tok) + 4 * D, T * D, g * D, D, 0, S())
    t = tok.view(N, T, D).cpu()
    assert torch.all(t[:, 0] == 9.0)
    _close(t[:, 1:].reshape(N, g, g, D), _nhwc(F.conv2d(_bf(x.double()), _bf(w.double()), stride=k)), atol=2e-5)
    C2 = 64
    w2 = torch.randn(C2, D, 1, 1) * 0.1
    wp2 = torch.empty(C2 * D, dtype=torch.bfloat16, device=DEV)
    wt2 = torch.empty(C2 * D, dtype=torch.bfloat16, device=DEV)
    call("es_conv2d_pack_bf16", ptr(dv(w2)), C2, D, 1, 1, ptr(wp2), ptr(wt2), S())
    out = torch.empty(N, g, g, C2, device=DEV)
    call("es_conv2d_fwd_bf16", ptr(tok) + 4 * D, N, g, g, D, T * D, g * D, D, 1, ptr(wp2), None, C2, 1, 1, 1, 0,
         ptr(out), g * g * C2, g * C2, C2, 0, S())
    xin = _nchw(t[:, 1:].reshape(N, g, g, D)).double()
    _close(_nchw(out.cpu()), F.conv2d(_bf(xin), _bf(w2.double())), atol=2e-5)
    dy = torch.randn(N, g, g, C2)
    dtok = torch.zeros(N * T, D, device=DEV)
    call("es_conv2d_bwd_data_bf16", ptr(dv(dy)), g * g * C2, g * C2, C2, ptr(wt2), N, g, g, D, C2, 1, 1, 1, 0,
         ptr(dtok) + 4 * D, T * D, g * D, D, 1, 0, S())
    ref = torch.einsum("nhwo,oc->nhwc", _bf(dy.double()), _bf(w2.double()).view(C2, D))
    d = dtok.view(N, T, D).cpu()
    assert torch.all(d[:, 0] == 0)
    _close(d[:, 1:].reshape(N, g, g, D), ref, atol=2e-5)


def test_conv2d_strided_views():
    """NCHW image input (the stem) and token-row output / input (trans_patch_conv, FCUUp)."""
    torch.manual_seed(3)
    N, Cin, H, Cout, k = 2, 3, 20, 8, 4
    T = (H // k) ** 2 + 1
    x = torch.randn(N, Cin, H, H)
    w = torch.randn(Cout, Cin, k, k) * 0.2
    y = F.conv2d(x.double(), w.double(), stride=k)  # [N, Cout, 5, 5]
    g = H // k
    xd, wd = x.to(DEV), w.to(DEV)
    tok = torch.full((N * T, Cout), 9.0, device=DEV)
    call("es_conv2d_fwd", ptr(xd), N, H, H, Cin, Cin * H * H, H, 1, H * H, ptr(wd), None, Cout, k, k, k, 0,
         ptr(tok) + 4 * Cout, T * Cout, g * Cout, Cout, 0, S())
    t = tok.view(N, T, Cout).cpu()
    assert torch.all(t[:, 0] == 9.0)
    _close(t[:, 1:].reshape(N, g, g, Cout), _nhwc(y))
    # token rows read back as an NHWC map by a 1x1 conv, data gradient written into token rows
    w2 = torch.randn(5, Cout, 1, 1) * 0.3
    y2 = F.conv2d(_nchw(t[:, 1:].reshape(N, g, g, Cout)).double(), w2.double())
    out = torch.empty(N, g, g, 5, device=DEV)
    call("es_conv2d_fwd", ptr(tok) + 4 * Cout, N, g, g, Cout, T * Cout, g * Cout, Cout, 1, ptr(dv(w2)), None, 5,
         1, 1, 1, 0, ptr(out), g * g * 5, g * 5, 5, 0, S())
    _close(_nchw(out.cpu()), y2)
    dy = torch.randn(N, g, g, 5)
    dtok = torch.zeros(N * T, Cout, device=DEV)
    call("es_conv2d_bwd_data", ptr(dv(dy)), g * g * 5, g * 5, 5, ptr(dv(w2)), N, g, g, Cout, 5, 1, 1, 1, 0,
         ptr(dtok) + 4 * Cout, T * Cout, g * Cout, Cout, 1, 0, S())
    ref = torch.einsum("nhwo,oc->nhwc", dy.double(), w2.double().view(5, Cout))
    d = dtok.view(N, T, Cout).cpu()
    assert torch.all(d[:, 0] == 0)
    _close(d[:, 1:].reshape(N, g, g, Cout), ref)


# ------------------------------------------------------------------------------------ batchnorm
@pytest.mark.parametrize("rows_shape,C,relu,with_res", [((4, 6, 6), 16, True, False), ((3, 5, 5), 64, False, True),
                                                        ((2, 3, 3), 300, True, True), ((64, 14, 14), 32, True, False),
                                                        ((8, 96, 96), 64, True, True), ((2, 40, 40), 18, False, False)])
def test_bn2d_fwd_bwd(rows_shape, C, relu, with_res):
    torch.manual_seed(C)
    N, H, W = rows_shape
    x = torch.randn(N, H, W, C, dtype=torch.float64) * 1.5 + 0.3
    res = torch.randn(N, H, W, C, dtype=torch.float64) if with_res else None
    g = 1 + 0.1 * torch.randn(C, dtype=torch.float64)
    b = 0.1 * torch.randn(C, dtype=torch.float64)
    rm, rv = 0.1 * torch.randn(C, dtype=torch.float64), 1 + torch.rand(C, dtype=torch.float64)
    rm_r, rv_r = rm.clone(), rv.clone()
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, g, b))
    resr = res.clone().requires_grad_(True) if with_res else None
    y = F.batch_norm(_nchw(xr), rm_r, rv_r, gr, br, training=True, momentum=0.1, eps=1e-6)
    y = _nhwc(y)
    if with_res:
        y = y + resr
    if relu:
        y = F.relu(y)
    rows = N * H * W
    f = dv
    xd, gd, bdv, rmd, rvd = f(x), f(g), f(b), f(rm), f(rv)
    resd = f(res) if with_res else None
    yd, mean, rstd = torch.empty_like(xd), torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    ws = torch.empty(_lib.load().es_chan_workspace(rows, C), device=DEV)
    call("es_bn2d_fwd", ptr(xd), rows, C, ptr(gd), ptr(bdv), ptr(rmd), ptr(rvd), ptr(nbt), 0.1, 1e-6, 1, ptr(resd),
         int(relu), ptr(yd), ptr(mean), ptr(rstd), ptr(ws), S())
    _close(yd.cpu(), y, atol=2e-5)
    _close(rmd.cpu(), rm_r, atol=1e-6)
    _close(rvd.cpu(), rv_r, atol=1e-5)
    assert int(nbt.item()) == 1
    dy = torch.randn_like(y)
    y.backward(dy)
    dx, gout = torch.empty_like(xd), torch.empty_like(xd) if with_res else None
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    call("es_bn2d_bwd", ptr(xd), ptr(yd), ptr(f(dy)), rows, C, int(relu), ptr(gd), ptr(mean), ptr(rstd), 1, ptr(rvd),
         1e-6, ptr(dx), ptr(gout), ptr(dg), ptr(db), 0, ptr(ws), S())
    _close(dx.cpu(), xr.grad, atol=2e-4)
    _close(dg.cpu(), gr.grad, atol=1e-4)
    _close(db.cpu(), br.grad, atol=1e-4)
    if with_res:
        _close(gout.cpu(), resr.grad, atol=1e-6)
    # eval mode: running statistics
    y2 = torch.empty_like(xd)
    call("es_bn2d_fwd", ptr(xd), rows, C, ptr(gd), ptr(bdv), ptr(rmd), ptr(rvd), None, 0.1, 1e-6, 0, None, 0, ptr(y2),
         None, None, None, S())
    ref = _nhwc(F.batch_norm(_nchw(x), rmd.cpu().double(), rvd.cpu().double(), g, b, training=False, eps=1e-6))
    _close(y2.cpu(), ref, atol=2e-5)


# ------------------------------------------------------------------------------------ bf16 maps
B16 = torch.bfloat16


def _rep(*shape, scale=1.0, shift=0.0):
    """fp32 values exactly representable in bf16 (so an fp32-map kernel and a bf16-map kernel read the
    same numbers)."""
    return (torch.randn(*shape, device=DEV) * scale + shift).to(B16).float()


@pytest.mark.parametrize("N,Cin,H,Cout,k,s,p", [(2, 64, 16, 64, 1, 1, 0), (3, 64, 15, 128, 3, 2, 1),
                                                (2, 32, 13, 96, 3, 1, 1)])
def test_conv_bf16_maps_match_fp32_maps_rounded(N, Cin, H, Cout, k, s, p):
    """es_conv2d_*_bf16_ex with bf16 maps: the same gathers, MFMAs and fp32 accumulation order as the fp32-map
    kernels, one rounding at the store -- so on bf16-representable inputs every bf16-map output is EXACTLY
    the fp32-map output rounded to bf16 (accumulating stores: the fp32 sum of the two, rounded), the weight
    gradient and the BatchNorm partials bit-identical, for every input / output dtype combination."""
    torch.manual_seed(N * 7 + Cin + Cout + k)
    lib = _lib.load()
    Ho = (H + 2 * p - k) // s + 1
    x32 = _rep(N, H, H, Cin)
    w = torch.randn(Cout, Cin, k, k, device=DEV) * 0.2
    b = torch.randn(Cout, device=DEV)
    n = Cout * Cin * k * k
    wp, wt = torch.empty(n, dtype=B16, device=DEV), torch.empty(n, dtype=B16, device=DEV)
    call("es_conv2d_pack_bf16", ptr(w), Cout, Cin, k, k, ptr(wp), ptr(wt), S())
    geo_x = (H * H * Cin, H * Cin, Cin)
    geo_y = (Ho * Ho * Cout, Ho * Cout, Cout)
    M = N * Ho * Ho
    prior = _rep(N, Ho, Ho, Cout)
    outs = {}
    for fx in (0, 1):
        for fy in (0, 1):
            xin = x32.to(B16) if fx else x32
            y = torch.empty(N, Ho, Ho, Cout, dtype=B16 if fy else torch.float32, device=DEV)
            part = torch.empty(lib.es_conv2d_bnstats_size(M, Cout), device=DEV)
            call("es_conv2d_fwd_bf16_ex", ptr(xin), N, H, H, Cin, *geo_x, 1, ptr(wp), ptr(b), Cout, k, k, s, p, ptr(y),
                 *geo_y, 0, ptr(part), fx | (fy << 1), S())
            ya = (prior.to(B16) if fy else prior.clone())
            call("es_conv2d_fwd_bf16_ex", ptr(xin), N, H, H, Cin, *geo_x, 1, ptr(wp), ptr(b), Cout, k, k, s, p, ptr(ya),
                 *geo_y, 1, None, fx | (fy << 1), S())
            outs[(fx, fy)] = (y, part, ya)
    y0, part0, ya0 = outs[(0, 0)]
    for (fx, fy), (y, part, ya) in outs.items():
        assert torch.equal(part, part0), (fx, fy)
        assert torch.equal(y.float(), y0.to(y.dtype).float()), (fx, fy)
        assert torch.equal(ya.float(), ya0.to(ya.dtype).float()), (fx, fy)
    # data gradient (dy -> dx) and weight gradient (x, dy)
    dy32 = _rep(N, Ho, Ho, Cout)
    dxp = _rep(N, H, H, Cin)
    dxs, dws = {}, {}
    for fa in (0, 1):
        for fb in (0, 1):
            dyin = dy32.to(B16) if fa else dy32
            dx = dxp.to(B16) if fb else dxp.clone()
            call("es_conv2d_bwd_data_bf16_ex", ptr(dyin), *geo_y, ptr(wt), N, H, H, Cin, Cout, k, k, s, p, ptr(dx),
                 *geo_x, 1, 1, fa | (fb << 1), S())
            dxs[(fa, fb)] = dx
            xin = x32.to(B16) if fa else x32
            dyw = dy32.to(B16) if fb else dy32
            ws = torch.empty(lib.es_conv2d_bwd_weight_bf16_workspace(M, Cout, Cin, k, k, 0), device=DEV)
            dw = torch.empty(Cout, Cin, k, k, device=DEV)
            call("es_conv2d_bwd_weight_bf16_ex", ptr(xin), N, H, H, Cin, *geo_x, 1, ptr(dyw), *geo_y, Cout, k, k, s, p,
                 0, ptr(ws), ptr(dw), 0, fa | (fb << 1), S())
            dws[(fa, fb)] = dw
    for key in dxs:
        assert torch.equal(dxs[key].float(), dxs[(0, 0)].to(dxs[key].dtype).float()), key
        assert torch.equal(dws[key], dws[(0, 0)]), key


@pytest.mark.parametrize("C,fl", [(64, 0), (64, 1), (256, 1), (6, 0), (6, 1)])
def test_bn_bwd_recompute_matches_bwd_with_y(C, fl):
    """es_bn2d_bwd_recompute_ex (the ReLU mask rebuilt from x with the forward's affine map and rounding, y not
    read) against es_bn2d_bwd_ex given the forward's y: dx, dgamma, dbeta bit-identical, fp32 and bf16 maps,
    vector (C % 4 == 0) and scalar kernels; x includes values on which the affine map lands at 0 and just
    beside it, where a mask that differed from the forward's would show."""
    torch.manual_seed(C + 17 * fl)
    N, H, W = 3, 9, 7
    rows = N * H * W
    lib = _lib.load()
    x = _rep(N, H, W, C, scale=1.5, shift=0.1)
    dy = _rep(N, H, W, C)
    g, b = 1 + 0.1 * torch.randn(C, device=DEV), 0.1 * torch.randn(C, device=DEV)
    if fl:
        x, dy = x.to(B16), dy.to(B16)
    ws = torch.empty(lib.es_chan_workspace(rows, C), device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    y, mean, rstd = torch.empty_like(x), torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    call("es_bn2d_fwd_ex", ptr(x), rows, C, ptr(g), ptr(b), ptr(rm), ptr(rv), None, 0.1, 1e-6, 1, None, 1, ptr(y),
         ptr(mean), ptr(rstd), ptr(ws), fl, S())
    # put every 5th row where the first pass's affine map is 0 (x = mean - beta / (rstd gamma), rounded), then
    # take the statistics and y of the edited map: those rows sit at the ReLU's edge
    x.view(rows, C)[::5] = (mean - b / (rstd * g)).to(x.dtype)
    call("es_bn2d_fwd_ex", ptr(x), rows, C, ptr(g), ptr(b), ptr(rm), ptr(rv), None, 0.1, 1e-6, 1, None, 1, ptr(y),
         ptr(mean), ptr(rstd), ptr(ws), fl, S())
    out = {}
    for mode in ("y", "recompute"):
        dx = torch.empty_like(x)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        if mode == "y":
            call("es_bn2d_bwd_ex", ptr(x), ptr(y), ptr(dy), rows, C, 1, ptr(g), ptr(mean), ptr(rstd), 1, ptr(rv),
                 1e-6, ptr(dx), None, ptr(dg), ptr(db), 0, ptr(ws), fl, S())
        else:
            call("es_bn2d_bwd_recompute_ex", ptr(x), ptr(dy), rows, C, ptr(g), ptr(b), ptr(mean), ptr(rstd), ptr(dx),
                 ptr(dg), ptr(db), 0, ptr(ws), fl, S())
        out[mode] = (dx, dg, db)
    for a, c in zip(out["y"], out["recompute"]):
        assert torch.equal(a, c)
    assert (y.float() == 0).any() and (y.float() > 0).any()


@pytest.mark.parametrize("C,fl,relu,with_res", [(64, 1, 1, 1), (256, 1, 1, 0), (768, 1, 0, 0), (96, 0, 1, 1),
                                                (512, 0, 1, 0), (12, 1, 1, 1)])
def test_bn_channel_stationary_bit_identical(C, fl, relu, with_res):
    """es_set_bn_cs: the channel-stationary BatchNorm apply kernels (forward apply; the backward's dx / gout pass,
    with y and with the ReLU mask rebuilt from x) against the per-iteration forms: every output BIT-identical, bf16
    (16-byte groups of 8) and fp32 maps, C a multiple of 8 / 4 or not (the fallback)."""
    torch.manual_seed(C + fl)
    N, H, W = 3, 11, 9
    rows = N * H * W
    lib = _lib.load()
    dt = B16 if fl else torch.float32
    x, dy = _rep(N, H, W, C, scale=1.5, shift=0.1).to(dt), _rep(N, H, W, C).to(dt)
    res = _rep(N, H, W, C).to(dt) if with_res else None
    g, b = 1 + 0.1 * torch.randn(C, device=DEV), 0.1 * torch.randn(C, device=DEV)
    ws = torch.empty(lib.es_chan_workspace(rows, C), device=DEV)
    out = {}
    try:
        for cs in (0, 1):
            assert lib.es_set_bn_cs(cs) in (0, 1)
            rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
            y, mean, rstd = torch.empty_like(x), torch.empty(C, device=DEV), torch.empty(C, device=DEV)
            call("es_bn2d_fwd_ex", ptr(x), rows, C, ptr(g), ptr(b), ptr(rm), ptr(rv), None, 0.1, 1e-6, 1,
                 ptr(res) if res is not None else None, relu, ptr(y), ptr(mean), ptr(rstd), ptr(ws), fl, S())
            ye = torch.empty_like(x)  # eval mode: rstd from the running variance inside the apply
            call("es_bn2d_fwd_ex", ptr(x), rows, C, ptr(g), ptr(b), ptr(rm), ptr(rv), None, 0.1, 1e-6, 0,
                 ptr(res) if res is not None else None, relu, ptr(ye), None, None, None, fl, S())
            dx, gout = torch.empty_like(x), torch.empty_like(x)
            dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
            call("es_bn2d_bwd_ex", ptr(x), ptr(y), ptr(dy), rows, C, relu, ptr(g), ptr(mean), ptr(rstd), 1, ptr(rv),
                 1e-6, ptr(dx), ptr(gout), ptr(dg), ptr(db), 0, ptr(ws), fl, S())
            got = [y, ye, dx, gout, dg, db]
            if relu and not with_res:
                dx2 = torch.empty_like(x)
                dg2, db2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
                call("es_bn2d_bwd_recompute_ex", ptr(x), ptr(dy), rows, C, ptr(g), ptr(b), ptr(mean), ptr(rstd),
                     ptr(dx2), ptr(dg2), ptr(db2), 0, ptr(ws), fl, S())
                got += [dx2, dg2, db2]
            torch.cuda.synchronize()
            out[cs] = [t.clone() for t in got]
    finally:
        lib.es_set_bn_cs(1)
    names = ["y", "y_eval", "dx", "gout", "dgamma", "dbeta", "dx_recompute", "dgamma_recompute", "dbeta_recompute"]
    for name, a, c in zip(names, out[1], out[0]):
        assert torch.equal(a, c), (name, (a.float() - c.float()).abs().max().item())


@pytest.mark.parametrize("relu,with_res,C", [(True, True, 64), (True, False, 256), (False, False, 128), (True, True, 6)])
def test_bn_pool_bf16_maps_match_fp32_maps_rounded(relu, with_res, C):
    """BatchNorm (statistics pass, conv partials, eval, backward, SyncBatchNorm halves), channel sums, max /
    average pooling and the nearest upsample-add over bf16 maps: fp32 arithmetic on the widened values, each
    output rounded once -- on bf16-representable inputs exactly the fp32-map kernels' outputs rounded."""
    torch.manual_seed(C + relu)
    N, H, W = 2, 12, 10
    rows = N * H * W
    lib = _lib.load()
    x32 = _rep(N, H, W, C, scale=1.5, shift=0.3)
    res32 = _rep(N, H, W, C) if with_res else None
    dy32 = _rep(N, H, W, C)
    g, b = 1 + 0.1 * torch.randn(C, device=DEV), 0.1 * torch.randn(C, device=DEV)
    ws = torch.empty(lib.es_chan_workspace(rows, C), device=DEV)
    res_ = {}
    for fl in (0, 1):
        cv = (lambda t: None if t is None else t.to(B16)) if fl else (lambda t: t)
        x, res, dy = cv(x32), cv(res32), cv(dy32)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        nbt = torch.zeros((), dtype=torch.int64, device=DEV)
        y, mean, rstd = torch.empty_like(x), torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        call("es_bn2d_fwd_ex", ptr(x), rows, C, ptr(g), ptr(b), ptr(rm), ptr(rv), ptr(nbt), 0.1, 1e-6, 1, ptr(res),
             int(relu), ptr(y), ptr(mean), ptr(rstd), ptr(ws), fl, S())
        ye = torch.empty_like(x)
        call("es_bn2d_fwd_ex", ptr(x), rows, C, ptr(g), ptr(b), ptr(rm), ptr(rv), None, 0.1, 1e-6, 0, ptr(res),
             int(relu), ptr(ye), None, None, None, fl, S())
        dx, gout = torch.empty_like(x), torch.empty_like(x)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        call("es_bn2d_bwd_ex", ptr(x), ptr(y), ptr(dy), rows, C, int(relu), ptr(g), ptr(mean), ptr(rstd), 1, ptr(rv),
             1e-6, ptr(dx), ptr(gout), ptr(dg), ptr(db), 0, ptr(ws), fl, S())
        sums = torch.empty(2, C, device=DEV)
        call("es_bn2d_sums_ex", ptr(x), rows, C, 0, None, 0, ptr(sums[0]), ptr(ws), fl, S())
        call("es_bn2d_sums_ex", ptr(x), rows, C, 1, ptr(sums[0]), rows, ptr(sums[1]), ptr(ws), fl, S())
        yg, mg, rg = torch.empty_like(x), torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        call("es_bn2d_fwd_global_ex", ptr(x), rows, C, ptr(g), ptr(b), ptr(rm2), ptr(rv2), None, 0.1, 1e-6,
             ptr(sums[0]), ptr(sums[1]), rows, ptr(res), int(relu), ptr(yg), ptr(mg), ptr(rg), fl, S())
        loc = torch.empty(2 * C, device=DEV)
        call("es_bn2d_bwd_sums_ex", ptr(x), ptr(yg), ptr(dy), rows, C, int(relu), ptr(mg), ptr(rg), ptr(loc), ptr(ws),
             fl, S())
        dxg, dg2, db2 = torch.empty_like(x), torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        call("es_bn2d_bwd_global_ex", ptr(x), ptr(yg), ptr(dy), rows, C, int(relu), ptr(g), ptr(mg), ptr(rg), ptr(loc),
             ptr(loc), rows, ptr(dxg), None, ptr(dg2), ptr(db2), 0, fl, S())
        cs = torch.empty(C, device=DEV)
        call("es_chan_sum_ex", ptr(dy), rows, C, rows * C, C, rows, ptr(ws), ptr(cs), 0, fl, S())
        out = {"y": y, "ye": ye, "dx": dx, "gout": gout, "yg": yg, "dxg": dxg, "mean": mean, "rstd": rstd, "rm": rm,
               "rv": rv, "dg": dg, "db": db, "loc": loc, "dg2": dg2, "db2": db2, "cs": cs}
        res_[fl] = out
    for k, v1 in res_[1].items():
        v0 = res_[0][k]
        assert torch.equal(v1.float(), v0.to(B16).float() if v1.dtype == B16 else v0), k
    if C % 4:
        return
    # pools / upsampling (bf16 maps always have C % 4 == 0), stage by stage: each bf16-map kernel against the
    # fp32-map kernel fed the same (widened) inputs, rounded
    H2, W2 = H // 2, W // 2
    x16 = x32.to(B16)

    def both(name, mk_out, args16, args32, flags):
        o16, o32 = mk_out(B16), mk_out(torch.float32)
        call(name + "_ex", *args16(o16), flags, S())
        call(name, *args32(o32), S())
        return o16, o32

    yp16, yp32 = both("es_avgpool2d_fwd", lambda dt: torch.empty(N, H2, W2, C, dtype=dt, device=DEV),
                      lambda o: (ptr(x16), N, H, W, C, 2, ptr(o)), lambda o: (ptr(x32), N, H, W, C, 2, ptr(o)), 3)
    assert torch.equal(yp16.float(), yp32.to(B16).float())
    ypw = yp16.float()
    dxp32 = _rep(N, H, W, C)
    d16, d32 = dxp32.to(B16), dxp32.clone()
    call("es_avgpool2d_bwd_ex", ptr(yp16), N, H, W, C, 2, ptr(d16), 1, 3, S())
    call("es_avgpool2d_bwd", ptr(ypw), N, H, W, C, 2, ptr(d32), 1, S())
    assert torch.equal(d16.float(), d32.to(B16).float())
    up16, up32 = both("es_upsample_add_fwd", lambda dt: torch.empty(N, H, W, C, dtype=dt, device=DEV),
                      lambda o: (ptr(x16), ptr(yp16), N, H, W, C, 2, ptr(o)),
                      lambda o: (ptr(x32), ptr(ypw), N, H, W, C, 2, ptr(o)), 1)
    assert torch.equal(up16.float(), up32.to(B16).float())
    upw = up16.float()
    ds16, ds32 = both("es_upsample_bwd", lambda dt: torch.empty(N, H2, W2, C, dtype=dt, device=DEV),
                      lambda o: (ptr(up16), N, H, W, C, 2, ptr(o)), lambda o: (ptr(upw), N, H, W, C, 2, ptr(o)), 1)
    assert torch.equal(ds16.float(), ds32.to(B16).float())
    Hm, Wm = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    a16, a32 = (torch.empty(N, Hm, Wm, C, dtype=torch.int8, device=DEV) for _ in range(2))
    mp16, mp32 = both("es_maxpool2d_fwd", lambda dt: torch.empty(N, Hm, Wm, C, dtype=dt, device=DEV),
                      lambda o: (ptr(x32), N, H, W, C, 3, 2, 1, ptr(o), ptr(a16)),
                      lambda o: (ptr(x32), N, H, W, C, 3, 2, 1, ptr(o), ptr(a32)), 2)
    assert torch.equal(mp16.float(), mp32.to(B16).float()) and torch.equal(a16, a32)
    mpw = mp16.float()
    dm16, dm32 = torch.empty(N, H, W, C, device=DEV), torch.empty(N, H, W, C, device=DEV)
    call("es_maxpool2d_bwd_ex", ptr(mp16), ptr(a16), N, H, W, C, 3, 2, 1, ptr(dm16), 1, S())
    call("es_maxpool2d_bwd", ptr(mpw), ptr(a32), N, H, W, C, 3, 2, 1, ptr(dm32), S())
    assert torch.equal(dm16, dm32)


# ------------------------------------------------------------------------------------ pools
@pytest.mark.parametrize("C", [24, 6])  # the 4-channel vector kernels, and the scalar ones
def test_maxpool_avgpool_upsample(C):
    torch.manual_seed(11)
    N, H = 3, 13
    x = torch.randn(N, C, H, H, dtype=torch.float64)
    x[0, 0, 2, 2] = x[0, 0, 2, 3] = 5.0  # a tie inside one window: the first (row-major) wins, as torch
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 3, 2, 1)
    Ho = y.shape[2]
    xd = _nhwc(x).float().to(DEV)
    yd = torch.empty(N, Ho, Ho, C, device=DEV)
    arg = torch.empty(N, Ho, Ho, C, dtype=torch.int8, device=DEV)
    call("es_maxpool2d_fwd", ptr(xd), N, H, H, C, 3, 2, 1, ptr(yd), ptr(arg), S())
    _close(_nchw(yd.cpu()), y, atol=1e-6)
    dy = torch.randn_like(y)
    y.backward(dy)
    dxd = torch.empty_like(xd)
    call("es_maxpool2d_bwd", ptr(dv(_nhwc(dy))), ptr(arg), N, H, H, C, 3, 2, 1, ptr(dxd), S())
    _close(_nchw(dxd.cpu()), xr.grad, atol=1e-6)
    # avgpool k x k / k and the global pool
    for k, Hh in ((4, 16), (7, 7)):
        z = torch.randn(N, C, Hh, Hh, dtype=torch.float64, requires_grad=True)
        yz = F.avg_pool2d(z, k, k)
        zd = _nhwc(z.detach()).float().to(DEV)
        out = torch.empty(N, Hh // k, Hh // k, C, device=DEV)
        call("es_avgpool2d_fwd", ptr(zd), N, Hh, Hh, C, k, ptr(out), S())
        _close(_nchw(out.cpu()), yz, atol=1e-6)
        dyz = torch.randn_like(yz)
        yz.backward(dyz)
        dz = torch.empty_like(zd)
        call("es_avgpool2d_bwd", ptr(dv(_nhwc(dyz))), N, Hh, Hh, C, k, ptr(dz), 0, S())
        _close(_nchw(dz.cpu()), z.grad, atol=1e-6)
    # base + nearest upsample x s
    base = torch.randn(N, C, 12, 12, dtype=torch.float64, requires_grad=True)
    src = torch.randn(N, C, 3, 3, dtype=torch.float64, requires_grad=True)
    o = base + F.interpolate(src, size=(12, 12))
    od = torch.empty(N, 12, 12, C, device=DEV)
    call("es_upsample_add_fwd", ptr(dv(_nhwc(base.detach()))), ptr(dv(_nhwc(src.detach()))),
         N, 12, 12, C, 4, ptr(od), S())
    _close(_nchw(od.cpu()), o, atol=1e-6)
    do = torch.randn_like(o)
    o.backward(do)
    ds = torch.empty(N, 3, 3, C, device=DEV)
    call("es_upsample_bwd", ptr(dv(_nhwc(do))), N, 12, 12, C, 4, ptr(ds), S())
    _close(_nchw(ds.cpu()), src.grad, atol=1e-5)


@pytest.mark.parametrize("N,np_,D", [(5, 16, 128), (3, 4, 100), (260, 16, 384)])
def test_fcu_down_tokens_fwd_bwd(N, np_, D):
    """FCUDown LN + GELU + cat(cls) fused with `x_st + x_t` (code/models/conformer.py:161-170,345).
    (260, 16, 384): more rows than one pass of the 1024 backward workgroups, Conformer-Ti's D."""
    torch.manual_seed(21)
    T = np_ + 1
    pooled = torch.randn(N, np_, D, dtype=torch.float64) * 2 + 0.5
    xt = torch.randn(N, T, D, dtype=torch.float64)
    g = 1 + 0.1 * torch.randn(D, dtype=torch.float64)
    b = 0.1 * torch.randn(D, dtype=torch.float64)
    pr, xr, gr, br = (t.clone().requires_grad_(True) for t in (pooled, xt, g, b))
    xs = torch.cat([xr[:, 0][:, None, :], F.gelu(F.layer_norm(pr, (D,), gr, br, 1e-6))], dim=1)
    out = xs + xr
    f = dv
    od = torch.zeros(N * T, D, device=DEV)
    mean, rstd = torch.empty(N * np_, device=DEV), torch.empty(N * np_, device=DEV)
    call("es_fcu_down_tokens_fwd", ptr(f(pooled)), ptr(f(xt)), ptr(f(g)), ptr(f(b)), ptr(od), ptr(mean), ptr(rstd), N,
         np_, D, 1e-6, S())
    _close(od.view(N, T, D).cpu(), out, atol=2e-5)
    dout = torch.randn_like(out)
    out.backward(dout)
    dxt, dp = torch.empty(N * T, D, device=DEV), torch.empty(N, np_, D, device=DEV)
    dg, db = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    ws = torch.empty(_lib.load().es_fcu_down_workspace(N, np_, D), device=DEV)
    call("es_fcu_down_tokens_bwd", ptr(f(dout)), ptr(f(pooled)), ptr(f(g)), ptr(f(b)), ptr(mean), ptr(rstd), ptr(dxt),
         ptr(dp), ptr(dg), ptr(db), 0, N, np_, D, ptr(ws), S())
    _close(dxt.view(N, T, D).cpu(), xr.grad, atol=1e-5)
    _close(dp.cpu(), pr.grad, atol=1e-4)
    _close(dg.cpu(), gr.grad, atol=1e-4)
    _close(db.cpu(), br.grad, atol=1e-4)


def test_ce_weighted_fwd_bwd():
    torch.manual_seed(8)
    n, C = 37, 23
    lg = torch.randn(n, C, dtype=torch.float64) * 3
    y = torch.randint(0, C, (n,))
    w = torch.rand(C, dtype=torch.float64) + 0.5
    for weights in (w, None):
        lr = lg.clone().requires_grad_(True)
        loss = F.cross_entropy(lr, y, weight=weights)
        loss.backward()
        out = torch.zeros(1, device=DEV)
        dl = torch.empty(n, C, device=DEV)
        call("es_ce_weighted_fwd_bwd", ptr(dv(lg)), C, ptr(dv(y, torch.int64)),
             ptr(dv(weights)) if weights is not None else None, n, C, 1.0, ptr(dl), C, ptr(out), S())
        assert abs(out.item() - loss.item()) <= 1e-5 * max(1.0, loss.item())
        _close(dl.cpu(), lr.grad, atol=1e-6)


# ------------------------------------------------------------------------------------ model / trainer
def _tiny_cfgs():
    from endossl.conformer import ConformerConfig
    kw = dict(img_size=64, patch=16, base_channel=64, channel_ratio=1, embed_dim=128, depth=6, heads=2, num_classes=23)
    return ConformerConfig(**kw), cr.ConformerCfg(**kw)


def _model_from_fixture(d):
    from endossl.conformer import NativeConformer
    ncfg, _ = _tiny_cfgs()
    m = NativeConformer(ncfg, seed=0)
    state = {k[5:]: torch.tensor(d[k]) for k in d.files if k.startswith("init/")}
    m.load_state_dict(state)
    return m.to(DEV), state


@pytest.mark.parametrize("conv", ["fp32", "bf16"])
def test_conformer_forward_backward_vs_oracle(golden, conv):
    """One train-mode forward + backward of the native Conformer vs the oracle (bf16-contract mode:
    the transformer blocks' GEMM operands rounded like the MFMA kernels; with conv = "bf16" also the
    operands of the convs the device runs on conv_bf16.hip -- stages 2 and 3 of this fixture)."""
    d = golden("semiformer_step.npz")
    m, state = _model_from_fixture(d)
    m.set_conv_precision(conv)
    _, ocfg = _tiny_cfgs()
    x = torch.cat([torch.tensor(d[k]) for k in ("x0", "uw0", "us0")])
    _check_model_vs_oracle(m, state, ocfg, x, ("bn1.running_mean", "conv_trans_4.fusion_block.bn2.running_var",
                                              "conv_trans_6.expand_block.bn.running_mean"))


def test_conformer_vit_b_384_forward_backward_vs_oracle():
    """The SemiFormer stress shape (BASELINE configs[4]: a ViT-Base/16 transformer branch at 384^2):
    D = 768, 12 heads, T = 577 tokens (the long-sequence attention kernels, online softmax), on a
    CNN branch narrowed to base 16 channels and depth 3 so the CPU oracle finishes in seconds."""
    from endossl.conformer import ConformerConfig, NativeConformer
    kw = dict(img_size=384, patch=16, base_channel=16, channel_ratio=1, embed_dim=768, depth=3, heads=12,
              num_classes=23)
    ncfg, ocfg = ConformerConfig(**kw), cr.ConformerCfg(**kw)
    assert ncfg.T == 577
    m = NativeConformer(ncfg, seed=5)
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    x = torch.randn(3, 3, 384, 384, generator=torch.Generator().manual_seed(8))
    _check_model_vs_oracle(m, state, ocfg, x, ("bn1.running_mean", "conv_trans_2.fusion_block.bn2.running_var"))


def test_conformer_b_cnn_branch_bf16_vs_oracle():
    """Conformer-B's CNN branch (channel_ratio 4: stages of 256 / 512 / 1024 channels, bottlenecks of
    64 / 128 / 256) -- every conv but the stem on the bf16 kernels (csrc/conv_bf16.hip) -- at 64^2 so
    the CPU oracle stays fast; the oracle's bf16 mode rounds the same conv operands."""
    from endossl.conformer import ConformerConfig, NativeConformer
    kw = dict(img_size=64, patch=16, base_channel=64, channel_ratio=4, embed_dim=128, depth=3, heads=2,
              num_classes=23)
    ncfg, ocfg = ConformerConfig(**kw), cr.ConformerCfg(**kw)
    m = NativeConformer(ncfg, seed=11)
    assert m.conv_bf16
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    x = torch.randn(6, 3, 64, 64, generator=torch.Generator().manual_seed(12))
    _check_model_vs_oracle(m, state, ocfg, x, ("bn1.running_mean", "conv_trans_2.fusion_block.bn2.running_var",
                                              "conv_trans_3.cnn_block.bn1.running_mean"))


def test_bn_relu_fused_into_conv_gather_bit_identical():
    """conformer.BN_CONV_FUSED: a ConvBlock's bn1 -> conv2 and (x2 not returned) bn2 -> conv3 with the BatchNorm +
    ReLU applied by the bf16 conv's gathers (es_conv2d_fwd_bf16_bnin_ex / es_conv2d_bwd_weight_bf16_bnin_ex, the
    statistics-only es_bn2d_fwd_partials_ex, es_bn2d_bwd_recompute_ex) against the same ops with the normalised
    map written in between: logits, every parameter gradient and every BatchNorm running buffer BIT-identical
    over two train steps' forward + backward (Conformer-B's CNN branch, bf16 maps, strided 3x3 convs)."""
    from endossl import conformer as cf
    from endossl.conformer import ConformerConfig, NativeConformer
    kw = dict(img_size=64, patch=16, base_channel=64, channel_ratio=4, embed_dim=128, depth=3, heads=2, num_classes=23)
    saved = cf.BN_CONV_FUSED, cf.BN_CONV_FUSED_KXK
    res = {}
    calls = {}
    try:
        for fused in (False, True):
            cf.BN_CONV_FUSED = fused
            cf.BN_CONV_FUSED_KXK = True  # the 3 x 3 pairs too (off by default: measured slower)
            m = NativeConformer(ConformerConfig(**kw), seed=11).to(DEV)
            assert m.conv_bf16 and m.map_bf16
            m.train()
            g = torch.Generator().manual_seed(12)
            n_fused = [0]
            orig = cf._BNConvFn.apply

            def counting(*a, _o=orig, _n=n_fused):
                _n[0] += 1
                return _o(*a)
            cf._BNConvFn.apply = counting
            outs = []
            try:
                for _ in range(2):
                    x = torch.randn(6, 3, 64, 64, generator=g).to(DEV)
                    m.flat_grad.zero_()
                    oc, ot = m(x)
                    w = torch.randn(oc.shape, generator=g).to(DEV), torch.randn(ot.shape, generator=g).to(DEV)
                    (oc * w[0]).sum().add((ot * w[1]).sum()).backward()
                    torch.cuda.synchronize()
                    outs.append((oc.detach().clone(), ot.detach().clone(), m.flat_grad.clone(),
                                 {k: v.clone() for k, v in m.state_dict().items() if cr.is_buffer(k)}))
            finally:
                cf._BNConvFn.apply = orig
            res[fused], calls[fused] = outs, n_fused[0]
    finally:
        cf.BN_CONV_FUSED, cf.BN_CONV_FUSED_KXK = saved
    # conv_1's bn1 / bn2, each stage's cnn_block bn1 and fusion_block bn2 (fusion bn1 feeds the FCUUp add)
    nst = len(list(ConformerConfig(**kw).stages()))
    assert calls[False] == 0 and calls[True] == 2 * (2 + 2 * nst), calls
    for (a_oc, a_ot, a_g, a_b), (b_oc, b_ot, b_g, b_b) in zip(res[False], res[True]):
        assert torch.equal(a_oc, b_oc) and torch.equal(a_ot, b_ot)
        assert torch.equal(a_g, b_g), (a_g - b_g).abs().max().item()
        for k in a_b:
            assert torch.equal(a_b[k], b_b[k]), k


def _check_model_vs_oracle(m, state, ocfg, x, bn_keys):
    """Train-mode forward + backward vs the oracle in fp32 and in the device's bf16 contract.

    fp32 convs: the device tracks the contract emulation to within a quarter of the bf16 envelope
    (|contract - fp32|).  bf16 convs: the device rounds its OWN fp32 conv inputs, which differ from the
    emulation's in the last bits (summation order upstream); a rounding flip there is a bf16 ulp that
    the batch-statistics BatchNorms pass on, so the two bf16 computations are independent samples of
    the same error distribution.  The test then asks for the property that matters -- the device is as
    close to the fp32 reference as the contract emulation is: |device - fp32| <= 2 x envelope."""
    conv16 = m.conv_bf16
    rec = {"conv_bf16": conv16}
    res = {}
    for bf in (True, False):
        p = {k: v.clone().float().requires_grad_(True) for k, v in state.items() if not cr.is_buffer(k)}
        bufs = {k: v.clone() for k, v in state.items() if cr.is_buffer(k)}
        oc, ot = cr.conformer_forward(p, bufs, x, ocfg, train=True, bf16=bf, bf16_conv=bf and conv16,
                                      bf16_maps=bf and m.map_bf16)
        res[bf] = (oc, ot, p, bufs)
    m.train()
    m.flat_grad.zero_()
    hc, ht = m(x.to(DEV))
    for name, h, i in (("conv", hc, 0), ("trans", ht, 1)):
        r16, r32 = res[True][i].detach().double(), res[False][i].detach().double()
        sc = max(1.0, r32.abs().max().item())
        e16 = (h.detach().cpu().double() - r16).abs().max().item()
        e32 = (h.detach().cpu().double() - r32).abs().max().item()
        env = (r16 - r32).abs().max().item()
        rec[name] = {"hip_vs_bf16_contract": e16, "hip_vs_fp32": e32, "bf16_envelope": env, "scale": sc}
        if conv16:
            assert e32 <= 2 * env + 1e-3 * sc, rec
        else:
            assert e16 <= 1e-3 * sc + 0.25 * env, rec
    # BatchNorm running statistics after the train-mode forward
    for k in bn_keys:
        _close(m.get_buffer(k).cpu(), res[True][3][k], atol=2e-2 if conv16 else 2e-3)
    assert int(m.get_buffer("bn1.num_batches_tracked").item()) == int(state["bn1.num_batches_tracked"].item()) + 1
    # gradients of a fixed random linear functional of both heads
    g = torch.Generator().manual_seed(4)
    wc, wt = torch.randn(hc.shape, generator=g), torch.randn(ht.shape, generator=g)
    (hc * wc.to(DEV)).sum().add((ht * wt.to(DEV)).sum()).backward()
    grads = {}
    for bf in (True, False):
        oc, ot, p, _ = res[bf]
        ((oc * wc).sum() + (ot * wt).sum()).backward()
        grads[bf] = {k: v.grad for k, v in p.items()}
    # per tensor: |HIP - bf16 contract| <= 2e-3 |g| + |bf16 contract - fp32| (+ a floor at 1e-4 of the
    # largest gradient norm: a conv bias in front of a BatchNorm has an exactly-zero true gradient, so its
    # computed value is pure rounding noise in every arithmetic)
    gmax = max(grads[False][k].double().norm().item() for k in grads[False])
    worst, bad = [], []
    for k in grads[True]:
        gh = m.gview(k).cpu().view(grads[True][k].shape).double()
        g16, g32 = grads[True][k].double(), grads[False][k].double()
        nrm = g32.norm().item()
        e, env = (gh - g16).norm().item(), (g16 - g32).norm().item()
        if conv16:  # as the logits: the device within twice the contract's distance from fp32
            e = (gh - g32).norm().item()
            env = 2 * env
        worst.append((e / (nrm + 1e-12), env / (nrm + 1e-12), k))
        if e > 2e-3 * nrm + env + 1e-4 * gmax:
            bad.append((k, e, env, nrm))
    worst.sort(reverse=True)
    rec["worst_grad_rel"] = [(round(a, 6), round(b, 6), c) for a, b, c in worst[:8]]
    print(json.dumps(rec))
    assert not bad, bad[:8]


class _DL:
    def __init__(self, items, df=None):
        self.items = items

        class _DS:
            pass

        self.dataset = _DS()
        self.dataset.df = df

    def __iter__(self):
        return iter(self.items)

    def __len__(self):
        return len(self.items)


def _sf_loss_terms(oc, ot, y, bs, cw, pl, mask):
    """SemiFormer.train_one's loss terms (code/semiformer.py:120-131) recomputed in float64 from a pass's
    logits and the given pseudo-labels / mask: (lx, lu, per-row lx contributions of the labeled rows of both
    heads, per-row lu contributions of the strong rows of both heads), each row's share of the sum."""
    oc, ot, w = oc.double().cpu(), ot.double().cpu(), cw.double()
    nu = (oc.shape[0] - bs) // 2
    wy = w[y]
    rx = (F.cross_entropy(oc[:bs], y, reduction="none") + F.cross_entropy(ot[:bs], y, reduction="none")) * wy / wy.sum()
    m = mask.double().cpu()
    pl = pl.long().cpu()
    ru = (F.cross_entropy(oc[bs + nu:], pl, reduction="none") + F.cross_entropy(ot[bs + nu:], pl, reduction="none")) * m / nu
    return rx.sum().item(), ru.sum().item(), rx, ru


_SF_METRICS = {}


def _record_sf(key, rec):
    """Keep a trainer test's record in gpurun_out/semiformer_trainer_metrics.json (one key per case)."""
    import os
    _SF_METRICS[key] = rec
    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "semiformer_trainer_metrics.json"), "w") as f:
        json.dump(_SF_METRICS, f, indent=1, default=float)


@pytest.mark.parametrize("conv,sum8", [("fp32", 0), ("bf16", 0), ("bf16", 1)])
def test_semiformer_trainer_vs_reference_train_one(golden, conv, sum8):
    """The SemiFormer trainer over the fixture's steps (round 6 fixture: B = 4, mu = 7 -- 28 unlabeled rows,
    BatchNorm statistics over 60 images).  kc / kr / kd: the tolerance factors on the bf16 envelope; with bf16
    convs the device is an independent bf16 sample (see _check_model_vs_oracle), so it is held to the envelope
    itself rather than a fraction of it.  sum8: the BatchNorm channel sums in the other fp32 summation order
    (es_set_bn_sum8: 8-channel groups, round 5's reverted change) -- a legitimate reordering must pass the
    same bars."""
    import pandas as pd
    from endossl.semiformer import SemiFormer
    from endossl.utils import AttrDict
    lib = _lib.load()
    old_sum8 = lib.es_set_bn_sum8(sum8)
    try:
        _semiformer_trainer_vs_reference(golden, conv, sum8, pd, SemiFormer, AttrDict)
    finally:
        lib.es_set_bn_sum8(old_sum8)


def _semiformer_trainer_vs_reference(golden, conv, sum8, pd, SemiFormer, AttrDict):
    d = golden("semiformer_step.npz")
    m, state = _model_from_fixture(d)
    m.set_conv_precision(conv)
    c16 = conv == "bf16"
    kc, kr, kd = (2.0, 3.0, 4.0) if c16 else (0.25, 1.5, 2.0)
    _, ocfg = _tiny_cfgs()
    B, MU, steps, thres = int(d["B"]), int(d["MU"]), int(d["steps"]), float(d["thres"])
    C = 23
    df = pd.DataFrame({"target": np.concatenate([np.full(i + 1, i) for i in range(C)])})
    lab = [(torch.tensor(d[f"x{i}"]), torch.tensor(d[f"y{i}"])) for i in range(steps)]
    unl = [((torch.tensor(d[f"uw{i}"]), torch.tensor(d[f"us{i}"])), None) for i in range(steps)]
    tr = SemiFormer(m, opt_func="Adam", lr=1e-3, device=DEV)
    tr.get_dataloader((_DL(lab, df), _DL(unl)), None)
    tr.get_config(AttrDict(
        DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=64, TARGET_NAME="target"),
        MODEL=AttrDict(NAME="conformer", NUM_CLASSES=C),
        TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=steps, EVAL_STEP_SUP=0,
                       CLS_WEIGHT=True, THRES=thres, T=1.0, LAMBDA_U=1.0, EPOCHS=1, WARMUP_EPOCHS=0, DECAY_EPOCHS=10,
                       WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const", FREQ_EVAL=1)))
    np.testing.assert_allclose(tr.class_weights.cpu().numpy(), d["class_weights"], rtol=1e-6)
    cw = torch.tensor(d["class_weights"]).float()
    emu = cr.SemiFormerRef(state, ocfg, class_weights=cw, thres=thres, bf16=True, bf16_conv=c16, bf16_maps=m.map_bf16)
    rec = {}
    for i in range(steps):
        # the oracle at the HIP path's own pre-step state (parameters + BN buffers): every step is checked
        # tightly against the bf16-contract emulation of that state, not against a diverging trajectory
        # (Adam turns bf16 noise on near-zero gradients into +-lr moves, which BatchNorm then amplifies)
        snap = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        ref16 = cr.SemiFormerRef(snap, ocfg, class_weights=cw, thres=thres, bf16=True, bf16_conv=c16,
                                 bf16_maps=m.map_bf16)
        ref32 = cr.SemiFormerRef(snap, ocfg, class_weights=cw, thres=thres, bf16=False)
        o = tr.step((lab[i], unl[i]))
        r16, r32 = ref16.step(*lab[i], *unl[i][0]), ref32.step(*lab[i], *unl[i][0])
        r = emu.step(*lab[i], *unl[i][0])
        for head in ("out_conv", "out_trans"):
            h = o[head].cpu().double()
            a16, a32 = r16[head].double(), r32[head].double()
            sc = max(1.0, a32.abs().max().item())
            e, env = (h - a16).abs().max().item(), (a16 - a32).abs().max().item()
            rec[f"step{i}_{head}_vs_contract_at_hip_state"] = {"err": e, "bf16_envelope": env}
            assert e <= 1e-3 * sc + kc * env, rec
            if i == 0:  # same initial state as the reference fixture
                ref = torch.tensor(d[f"{head}{i}"]).double()
                err, envr = (h - ref).abs().max().item(), (r[head].double() - ref).abs().max().item()
                rec[f"step0_{head}_vs_reference"] = {"err": err, "bf16_envelope": envr}
                assert err <= kr * envr + 1e-3 * sc, rec
        # pseudo-labels / masks of the conv head's weak rows, on decidable rows of the fp32 oracle at
        # the same state (the reference's own at step 0)
        wk32 = r32["out_conv"][B:B + B * MU].double()
        wk16 = r16["out_conv"][B:B + B * MU].double()
        p32, p16 = torch.softmax(wk32, -1), torch.softmax(wk16, -1)
        envp = (p32 - p16).abs().max(-1).values  # per row: the contract's own distance from fp32 on that row
        top2 = p32.topk(2, -1).values
        ok = ((top2[:, 0] - top2[:, 1]) > kd * envp + 1e-6).numpy()
        okm = ((p32.max(-1).values - thres).abs() > kd * envp + 1e-6).numpy()
        hpl, hm = o["pseudo_label"].cpu(), o["mask"].cpu().to(torch.uint8)
        np.testing.assert_array_equal(hpl.numpy()[ok], r32["pseudo_label"].numpy()[ok])
        np.testing.assert_array_equal(hm.numpy().astype(bool)[okm], r32["mask"].numpy().astype(bool)[okm])
        # Losses.  lu is a masked mean, so a mask or pseudo-label decision on a row whose fp32 weak probability
        # sits within the envelope of tau (or of a tie) is a coin toss between any two bf16 evaluations and
        # moves lu by that row's whole CE / nu -- the contract's terms are therefore recomputed from its OWN
        # logits with the device's decisions on exactly those undecidable rows.  Bar (round 3's): |hip -
        # contract| <= 1e-3 max(1, |fp32|) + kc |contract - fp32| (difference of the sums, aligned decisions);
        # the record also keeps the L1 norm of the per-row differences, the per-row split and every flip.
        y_i = lab[i][1]
        pl16, m16 = r16["pseudo_label"].cpu().clone(), r16["mask"].cpu().to(torch.uint8).clone()
        und_l, und_m = torch.from_numpy(~ok), torch.from_numpy(~okm)
        pl16[und_l], m16[und_m] = hpl[und_l].to(pl16.dtype), hm[und_m]
        pl32, m32 = r32["pseudo_label"].cpu().clone(), r32["mask"].cpu().to(torch.uint8).clone()
        pl32[und_l], m32[und_m] = hpl[und_l].to(pl32.dtype), hm[und_m]
        lx_h, lu_h, rxh, ruh = _sf_loss_terms(o["out_conv"], o["out_trans"], y_i, B, cw, hpl, hm)
        lx_a, lu_a, rxa, rua = _sf_loss_terms(r16["out_conv"], r16["out_trans"], y_i, B, cw, pl16, m16)
        lx_f, lu_f, rxf, ruf = _sf_loss_terms(r32["out_conv"], r32["out_trans"], y_i, B, cw, pl32, m32)
        flips = [(j, int(hm[j]), int(r16["mask"][j]), int(hpl[j]), int(r16["pseudo_label"][j]),
                  round(float(p32.max(-1).values[j]), 6)) for j in range(len(hm))
                 if int(hm[j]) != int(r16["mask"][j]) or (int(hm[j]) and int(hpl[j]) != int(r16["pseudo_label"][j]))]
        rec[f"step{i}_rows"] = {"device_vs_contract_decision_flips(row,mask_h,mask_c,pl_h,pl_c,p32max)": flips,
                                "lu_rows_hip_minus_contract": [round(float(v), 7) for v in ruh - rua],
                                "lu_rows_contract_minus_fp32": [round(float(v), 7) for v in rua - ruf],
                                "lx_rows_hip_minus_contract": [round(float(v), 7) for v in rxh - rxa],
                                "lx_rows_contract_minus_fp32": [round(float(v), 7) for v in rxa - rxf]}
        # the device's reported losses are its own logits' losses (kernel vs float64 restatement)
        assert abs(o["lx"].item() - lx_h) <= 1e-4 * max(1.0, abs(lx_h)), rec
        assert abs(o["lu"].item() - lu_h) <= 1e-4 * max(1.0, abs(lu_h)), rec
        l1 = {"lx": (rxa - rxf).abs().sum().item(), "lu": (rua - ruf).abs().sum().item()}
        l1["loss"] = l1["lx"] + l1["lu"]
        for k, hip, a16, a32 in (("lx", lx_h, lx_a, lx_f), ("lu", lu_h, lu_a, lu_f),
                                 ("loss", lx_h + lu_h, lx_a + lu_a, lx_f + lu_f)):
            bar = 1e-3 * max(1.0, abs(a32)) + kc * abs(a16 - a32)
            rec[f"step{i}_{k}"] = {"hip": hip, "bf16_contract_aligned": a16, "fp32_aligned": a32,
                                   "bf16_contract": r16[k], "fp32": r32[k], "envelope": abs(a16 - a32),
                                   "row_l1_envelope": l1[k], "bar": bar}
            assert abs(hip - a16) <= bar, rec
        if i == 0:
            for k, ref_v in (("lx", float(d["lx"][0] + d["lx"][1])), ("lu", float(d["lu"][0] + d["lu"][1]))):
                assert abs(o[k].item() - ref_v) <= kr * abs(r[k] - ref_v) + 1e-3 * max(1.0, abs(ref_v)), rec
        if i == 0:
            np.testing.assert_array_equal(r32["pseudo_label"].numpy(), d["pseudo_label"][0])
        rec[f"step{i}_decidable"] = f"{int(ok.sum())}/{len(ok)} labels, {int(okm.sum())}/{len(okm)} masks"
        if i == 0:  # the fixture's tau keeps at least half the step-0 masks decidable (bf16 convs included)
            assert 2 * int(okm.sum()) >= len(okm), rec
    sd, esd = m.state_dict(), tr.ema_model.ema.state_dict()
    worst = 0.0
    for k, v in sd.items():
        if cr.is_buffer(k):
            if k.endswith("num_batches_tracked"):
                assert int(v.item()) == int(d["final/" + k])
                assert int(esd[k].item()) == int(d["ema/" + k])
            else:
                fx = torch.tensor(d["final/" + k])
                e, ev = (v.cpu() - fx).abs().max().item(), (emu.bufs[k] - fx).abs().max().item()
                assert e <= kr * ev + 2e-3, (k, e, ev)
            continue
        if "final/" + k in d.files:
            worst = max(worst, (v.cpu() - torch.tensor(d["final/" + k])).abs().max().item())
            assert (esd[k].cpu() - torch.tensor(d["ema/" + k])).abs().max().item() <= 1e-3 * 2e-3 * steps * (steps + 1) / 2 + 1e-6, k
        else:
            assert abs(v.double().sum().item() - float(d["final_sum/" + k])) <= (2e-3 * steps + 1e-5) * v.numel(), k
    rec["max_param_delta"] = worst
    print(json.dumps(rec))
    _record_sf(f"trainer_{conv}_sum{sum8}", rec)
    assert worst <= 2e-3 * steps + 1e-5


def test_conv_weight_grads_on_side_stream_match_serial(golden):
    """conformer.CONV_DW_SIDE: the conv and transformer-block weight / bias gradients run on a side
    HIP stream beside the data-gradient chain (block scratch double-buffered, event-ordered) and are
    joined by an autograd final callback.  Same kernels on the same inputs, so every conv / Linear
    gradient is bit-identical to the single-stream backward, and the rest of the flat gradient
    agrees within fp32 summation order (head atomics)."""
    from endossl import conformer as cf
    d = golden("semiformer_step.npz")
    m, _ = _model_from_fixture(d)
    x = torch.cat([torch.tensor(d[k]) for k in ("x0", "uw0", "us0")]).to(DEV)
    g = torch.Generator().manual_seed(7)
    m.train()
    grads, w = {}, None
    saved = cf.CONV_DW_SIDE
    try:
        for side in (False, True):
            cf.CONV_DW_SIDE = side
            m.flat_grad.zero_()
            hc, ht = m(x)
            if w is None:  # one fixed linear functional of both heads for both passes
                w = (torch.randn(hc.shape, generator=g).to(DEV), torch.randn(ht.shape, generator=g).to(DEV))
            (hc * w[0]).sum().add((ht * w[1]).sum()).backward()
            # read right after backward() returns, on the caller's stream: no explicit synchronize
            grads[side] = m.flat_grad.clone()
    finally:
        cf.CONV_DW_SIDE = saved
    conv_names = [n for n, _, k in m.layout if k == "p" and (".conv" in n or n.startswith("conv") or "conv_project" in n
                                                             or "residual_conv" in n or "trans_patch_conv" in n)]
    lin_names = [n for n, _, k in m.layout if k == "p" and (".attn." in n or ".mlp." in n)]
    assert len(conv_names) > 20 and len(lin_names) > 20
    for n in conv_names + lin_names:
        o, sh = m.offs[n], m.shapes[n]
        cnt = int(torch.tensor(sh).prod().item()) if len(sh) else 1
        assert torch.equal(grads[True][o:o + cnt], grads[False][o:o + cnt]), n
    torch.testing.assert_close(grads[True], grads[False], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("side", [True, False])
def test_block_weight_grads_grouped_match_per_linear(side):
    """conformer.CONF_TN_GROUPED: a transformer block's four weight gradients (fc2, fc1, proj, qkv) as one
    es_gemm_tn_big_grouped launch + reduce (384 x 192 tiles, split-K over the tokens) against the four
    es_gemm_tn launches -- D = 768, T = 577 (the S1 shape), on the side stream beside the branch streams and
    serial.  Same products, another split-K summation order: the Linear weight / bias gradients within fp32
    rounding of |g|, every other gradient (convs, LayerNorm, BatchNorm, tokens) bit-identical."""
    from endossl import conformer as cf
    from endossl.conformer import ConformerConfig, NativeConformer
    kw = dict(img_size=384, patch=16, base_channel=16, channel_ratio=1, embed_dim=768, depth=3, heads=12,
              num_classes=23)
    m = NativeConformer(ConformerConfig(**kw), seed=3).to(DEV)
    x = torch.randn(3, 3, 384, 384, generator=torch.Generator().manual_seed(4)).to(DEV)
    g = torch.Generator().manual_seed(5)
    m.train()
    grads, w = {}, None
    saved = cf.CONF_TN_GROUPED, cf.CONV_DW_SIDE
    try:
        cf.CONV_DW_SIDE = side
        for grouped in (False, True):
            cf.CONF_TN_GROUPED = grouped
            hc, ht = m(x)
            if w is None:
                w = (torch.randn(hc.shape, generator=g).to(DEV), torch.randn(ht.shape, generator=g).to(DEV))
            m.flat_grad.zero_()
            (hc * w[0]).sum().add((ht * w[1]).sum()).backward()
            grads[grouped] = m.flat_grad.clone()
    finally:
        cf.CONF_TN_GROUPED, cf.CONV_DW_SIDE = saved
    lin = [n for n, _, k in m.layout if k == "p" and (".attn.qkv." in n or ".attn.proj." in n or ".mlp." in n)]
    assert len(lin) == 24
    mask = torch.zeros_like(grads[True], dtype=torch.bool)
    for n in lin:
        o, sh = m.offs[n], m.shapes[n]
        cnt = int(torch.tensor(sh).prod().item())
        a, b = grads[True][o:o + cnt], grads[False][o:o + cnt]
        assert torch.isfinite(a).all(), n
        assert (a - b).abs().max().item() <= 2e-5 * b.abs().max().item() + 1e-7, n
        mask[o:o + cnt] = True
    assert torch.equal(grads[True][~mask], grads[False][~mask])
