"""Kernel-level parity on the MI355X: every C-ABI entry point against a plain fp32 reference of the
same op (torch on the same device, same bf16 inputs), plus exact-integer layout checks and the
reference-generated golden fixtures for the loss / EMA kernels."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402

DEV = "cuda"
EPI_BF16, EPI_GELU, EPI_F32_RESID, EPI_DGELU, EPI_F32, EPI_PATCH, EPI_GELU_ACT, EPI_GELU_D, EPI_MULAUX = range(9)


def S():
    return _lib.stream()


def _int_bf16(*shape, lo=-3, hi=4, gen=None):
    return torch.randint(lo, hi, shape, generator=gen, dtype=torch.int32).to(torch.bfloat16).to(DEV)


def _pad_rows(t, mult=256):
    M = t.shape[0]
    Mp = (M + mult - 1) // mult * mult
    out = torch.zeros((Mp,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    out[:M] = t
    return out


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    _lib.load()


# ------------------------------------------------------------------------------------- GEMM NT
# the NT kernel families es_gemm_nt's per-shape rules select (variant 1: the 256x128 BK64 kernel for long-K GEMMs)
GEMM_VARIANTS = [-1, 0, 1, 2, 5, 6, 10, 11]
_TILE_N = {6: 256, 10: 128}  # big-tile variants: N must be a multiple of the tile width


_LONG_M = (-1, 10)  # the families the rules pick for long token axes (the rest are tested at short M)


def _gemm_cases(shapes, n_of):
    """(variant, *shape) for every variant that tiles the shape's N (and, for M > 10,000, the long-axis
    families only): no runtime skips."""
    out = []
    for v in GEMM_VARIANTS:
        for sh in shapes:
            M, N = n_of(sh)
            if N % _TILE_N.get(v, 128) or (M > 10000 and v not in _LONG_M):
                continue
            out.append(pytest.param(v, *sh, id=f"v{v}-" + "-".join(map(str, sh))))
    return out


class _Pinned:
    """es_set_gemm_variant(v) for the duration of a test."""

    def __init__(self, v):
        self.v = v

    def __enter__(self):
        self.old = _lib.load().es_set_gemm_variant(self.v)

    def __exit__(self, *exc):
        _lib.load().es_set_gemm_variant(self.old)


@pytest.mark.parametrize("variant,M,N,K", _gemm_cases(
    [(300, 256, 192), (1000, 384, 384), (128, 128, 64), (5000, 1152, 1536), (600, 768, 320), (40000, 1152, 384),
     (33000, 384, 1536)], lambda sh: (sh[0], sh[1])))
def test_gemm_nt_exact_integers(variant, M, N, K):
    with _Pinned(variant):
        _gemm_nt_exact_integers(M, N, K)


def _gemm_nt_exact_integers(M, N, K):
    g = torch.Generator().manual_seed(M + N + K)
    A = _pad_rows(_int_bf16(M, K, gen=g))
    B = _int_bf16(N, K, gen=g)
    bias = torch.randint(-4, 5, (N,), generator=g).float().to(DEV)
    ref = A[:M].float() @ B.float().t() + bias
    C = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    call("es_gemm_nt", EPI_F32, ptr(A), K, ptr(B), K, ptr(bias), ptr(C), N, None, None, 0, M, N, K, 0, S())
    torch.cuda.synchronize()
    torch.testing.assert_close(C, ref, rtol=0, atol=0)
    Cb = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    call("es_gemm_nt", EPI_BF16, ptr(A), K, ptr(B), K, ptr(bias), ptr(Cb), N, None, None, 0, M, N, K, 0, S())
    torch.testing.assert_close(Cb.float(), ref.bfloat16().float(), rtol=0, atol=0)


@pytest.mark.parametrize("variant,N,M", _gemm_cases([(512, 777), (384, 777), (384, 70000), (1536, 30000)],
                                                   lambda sh: (sh[1], sh[0])))
def test_gemm_nt_epilogues_vs_fp32(variant, N, M):
    with _Pinned(variant):
        _gemm_nt_epilogues_vs_fp32(N, M)


def _gemm_nt_epilogues_vs_fp32(N, M):
    torch.manual_seed(0)
    K = 384
    A = _pad_rows(torch.randn(M, K, device=DEV).bfloat16())
    B = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N, device=DEV) * 0.1
    acc = A[:M].float() @ B.float().t() + bias
    # GELU: pre and act
    pre = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    act = torch.zeros_like(pre)
    call("es_gemm_nt", EPI_GELU, ptr(A), K, ptr(B), K, ptr(bias), ptr(pre), N, ptr(act), None, 0, M, N, K, 0, S())
    torch.testing.assert_close(pre.float(), acc, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(act.float(), F.gelu(acc), rtol=1e-2, atol=1e-2)
    # residual fp32
    res = torch.randn(M, N, device=DEV)
    out = torch.zeros(M, N, device=DEV)
    call("es_gemm_nt", EPI_F32_RESID, ptr(A), K, ptr(B), K, ptr(bias), ptr(out), N, None, ptr(res), N, M, N, K, 0,
         S())
    torch.testing.assert_close(out, acc + res, rtol=1e-5, atol=1e-4)
    # dgelu: acc(no bias) * gelu'(pre)
    xpre = torch.randn(M, N, device=DEV).bfloat16()
    dpre = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
    call("es_gemm_nt", EPI_DGELU, ptr(A), K, ptr(B), K, None, ptr(dpre), N, None, ptr(xpre), N, M, N, K, 0, S())
    xp = xpre.float().requires_grad_(True)
    F.gelu(xp).backward(torch.ones_like(xp))
    ref = (A[:M].float() @ B.float().t()) * xp.grad
    torch.testing.assert_close(dpre.float(), ref, rtol=2e-2, atol=2e-2)
    # GELU_D: gelu'(acc + bias) and the same activation bits as EPI_GELU; MULAUX: acc * aux
    gd = torch.zeros_like(pre)
    act2 = torch.zeros_like(pre)
    call("es_gemm_nt", EPI_GELU_D, ptr(A), K, ptr(B), K, ptr(bias), ptr(gd), N, ptr(act2), None, 0, M, N, K, 0, S())
    assert torch.equal(act2, act)
    ac = acc.clone().requires_grad_(True)
    F.gelu(ac).backward(torch.ones_like(ac))
    torch.testing.assert_close(gd.float(), ac.grad, rtol=1e-2, atol=1e-2)
    dmul = torch.zeros_like(pre)
    call("es_gemm_nt", EPI_MULAUX, ptr(A), K, ptr(B), K, None, ptr(dmul), N, None, ptr(gd), N, M, N, K, 0, S())
    ref = (A[:M].float() @ B.float().t()) * gd.float()
    torch.testing.assert_close(dmul.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("variant,D", _gemm_cases([(128,), (768,)], lambda sh: (48, sh[0])))
def test_gemm_nt_patch_epilogue(variant, D):
    with _Pinned(variant):
        _gemm_nt_patch_epilogue(D)


def _gemm_nt_patch_epilogue(D):
    torch.manual_seed(1)
    n, npch, K = 3, 16, 768
    M = n * npch
    A = _pad_rows(torch.randn(M, K, device=DEV).bfloat16())
    B = (torch.randn(D, K, device=DEV) * 0.02).bfloat16()
    bias = torch.randn(D, device=DEV)
    pos = torch.randn(npch + 1, D, device=DEV)
    x = torch.full((n * (npch + 1), D), 7.0, device=DEV)
    call("es_gemm_nt", EPI_PATCH, ptr(A), K, ptr(B), K, ptr(bias), ptr(x), D, None, ptr(pos), D, M, D, K, npch, S())
    ref = (A[:M].float() @ B.float().t() + bias).view(n, npch, D) + pos[1:]
    xv = x.view(n, npch + 1, D)
    torch.testing.assert_close(xv[:, 1:], ref, rtol=1e-5, atol=1e-4)
    assert torch.all(xv[:, 0] == 7.0)  # CLS rows untouched


@pytest.mark.parametrize("M,N", [(777, 384), (70000, 1152), (30000, 1536), (40, 384), (5, 1152)])
def test_gemm_ws_matches_tiled_bit_for_bit(M, N):
    """Variant 12, the weight-stationary K = 384 kernel (gemm_nt_ws_kernel, opt-in), against the per-shape
    default: each output is the same chain of 12 MFMAs in K order, so every epilogue it takes gives the same
    bits.  Three launches in a row check that the chunk-claim counters reset themselves; a second stream uses
    its own counter block."""
    torch.manual_seed(M + N)
    K = 384
    A = _pad_rows(torch.randn(M, K, device=DEV).bfloat16())
    B = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N, device=DEV) * 0.1

    def run(epi):
        two = epi in (EPI_GELU, EPI_GELU_D)
        dt = torch.float32 if epi == EPI_F32 else torch.bfloat16
        C = torch.full((M, N), float("nan"), dtype=dt, device=DEV)
        C2 = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV) if two else None
        call("es_gemm_nt", epi, ptr(A), K, ptr(B), K, ptr(bias), ptr(C), N, ptr(C2) if two else None, None, 0, M,
             N, K, 0, S())
        return C, C2

    for epi in (EPI_BF16, EPI_GELU, EPI_GELU_ACT, EPI_GELU_D, EPI_F32):
        ref, ref2 = run(epi)
        with _Pinned(12):
            outs = [run(epi) for _ in range(3)]
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                outs.append(run(epi))
            torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        for C, C2 in outs:
            assert torch.equal(C, ref), f"epilogue {epi}"
            if ref2 is not None:
                assert torch.equal(C2, ref2), f"epilogue {epi} (second output)"


@pytest.mark.parametrize("M", [777, 100864, 12608, 5, 40])
def test_gemm_resid_ln_matches_two_launches_bit_for_bit(M):
    """es_gemm_nt_resid_ln (the attention projection + residual + norm2 in one launch, D = 384) against
    es_gemm_nt(EPI_F32_RESID) followed by es_layernorm_fwd: x, h, mean and rstd bit for bit, every row written;
    repeated launches (self-resetting tile claims) and a second stream."""
    torch.manual_seed(M)
    D, eps = 384, 1e-6
    A = _pad_rows(torch.randn(M, D, device=DEV).bfloat16())
    W = (torch.randn(D, D, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(D, device=DEV) * 0.1
    xin = torch.randn(M, D, device=DEV)
    gamma = 1.0 + 0.1 * torch.randn(D, device=DEV)
    beta = 0.1 * torch.randn(D, device=DEV)

    def bufs():
        nan = float("nan")
        return (torch.full((M, D), nan, device=DEV), torch.full((M, D), nan, dtype=torch.bfloat16, device=DEV),
                torch.full((M,), nan, device=DEV), torch.full((M,), nan, device=DEV))

    x0, h0, m0, r0 = bufs()
    call("es_gemm_nt", EPI_F32_RESID, ptr(A), D, ptr(W), D, ptr(bias), ptr(x0), D, None, ptr(xin), D, M, D, D, 0, S())
    call("es_layernorm_fwd", ptr(x0), D, ptr(gamma), ptr(beta), ptr(h0), D, ptr(m0), ptr(r0), M, D, eps, S())
    outs = []
    for k in range(4):
        o = bufs()
        side = torch.cuda.Stream() if k == 3 else None
        if side is not None:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side) if side is not None else torch.cuda.stream(torch.cuda.current_stream()):
            call("es_gemm_nt_resid_ln", ptr(A), D, ptr(W), D, ptr(bias), ptr(o[0]), D, ptr(xin), D, ptr(gamma),
                 ptr(beta), ptr(o[1]), D, ptr(o[2]), ptr(o[3]), M, D, D, eps, S())
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)
        outs.append(o)
    torch.cuda.synchronize()
    for x, h, m, r in outs:
        assert torch.equal(x, x0) and torch.equal(h, h0) and torch.equal(m, m0) and torch.equal(r, r0)


def test_gemm_resid_ln_rejects_other_widths():
    z = torch.zeros(256, 768, device=DEV)
    rc = _lib.load().es_gemm_nt_resid_ln(ptr(z), 768, ptr(z), 768, None, ptr(z), 768, ptr(z), 768, ptr(z), ptr(z),
                                         ptr(z), 768, ptr(z), ptr(z), 64, 768, 768, 1e-6, S())
    assert rc == -1  # ES_BAD_SHAPE: only D = 384


# ------------------------------------------------------------------------------------- GEMM TN
@pytest.fixture(params=[-1, 0, 7], ids=["auto", "t0", "b7"])
def tn_variant(request):
    old = _lib.load().es_set_tn_variant(request.param)
    yield request.param
    _lib.load().es_set_tn_variant(old)


@pytest.mark.parametrize("M,N1,N2,splits", [(1000, 128, 256, 1), (1000, 384, 128, 5), (4096, 256, 384, 17),
                                            (3000, 128, 128, 2), (1000, 384, 192, 1), (5000, 1152, 384, 0),
                                            (3000, 384, 1536, 7), (2500, 768, 384, 3)])
def test_gemm_tn_exact_integers(M, N1, N2, splits, tn_variant):
    g = torch.Generator().manual_seed(M + splits)
    A1 = _pad_rows(_int_bf16(M, N1, lo=-2, hi=3, gen=g))
    A2 = _pad_rows(_int_bf16(M, N2, lo=-2, hi=3, gen=g))
    ref = A1[:M].float().t() @ A2[:M].float()
    ws = torch.empty(_lib.load().es_gemm_tn_workspace(N1, N2, splits), device=DEV)
    out = torch.full((N1, N2), 3.0, device=DEV)
    bias = torch.full((N1,), 5.0, device=DEV)
    call("es_gemm_tn", ptr(A1), N1, ptr(A2), N2, M, N1, N2, splits, ptr(ws), ptr(out), 0, ptr(bias), S())
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
    torch.testing.assert_close(bias, A1[:M].float().sum(0), rtol=0, atol=0)  # fused bias grad
    call("es_gemm_tn", ptr(A1), N1, ptr(A2), N2, M, N1, N2, splits, ptr(ws), ptr(out), 1, None, S())
    torch.testing.assert_close(out, 2 * ref, rtol=0, atol=0)


def test_gemm_tn_grouped_exact_integers():
    """es_gemm_tn_grouped: several weight-gradient GEMMs (different M, N1, N2, row strides, with and
    without the bias) in one launch, each tile over its whole token axis -- exact on integer data,
    outputs and biases overwritten."""
    import ctypes
    from endossl.vit import _TNProblem
    lib = _lib.load()
    assert lib.es_tn_problem_size() == ctypes.sizeof(_TNProblem) == 64
    g = torch.Generator().manual_seed(11)
    shapes = [(3008, 384, 1536, None), (3008, 1536, 384, None), (992, 1152, 384, None), (3008, 384, 384, 640),
              (64, 768, 384, None), (2000, 128, 128, None)]
    keep, tab, refs = [], (_TNProblem * len(shapes))(), []
    for e, (M, N1, N2, ld1) in zip(tab, shapes):
        ld1 = ld1 or N1
        A1 = _pad_rows(_int_bf16(M, ld1, lo=-2, hi=3, gen=g))
        A2 = _pad_rows(_int_bf16(M, N2, lo=-2, hi=3, gen=g))
        out = torch.full((N1, N2), 3.0, device=DEV)
        bias = torch.full((N1,), 5.0, device=DEV) if N1 != 128 else None
        keep += [A1, A2, out, bias]
        e.dy, e.x, e.out, e.bias_out = ptr(A1), ptr(A2), ptr(out), ptr(bias) if bias is not None else None
        e.M, e.N1, e.N2, e.ld1, e.ld2 = M, N1, N2, ld1, N2
        refs.append((out, bias, A1[:M, :N1].float().t() @ A2[:M].float(), A1[:M, :N1].float().sum(0)))
    tiles = lib.es_gemm_tn_grouped_prepare(ctypes.byref(tab), len(shapes))
    assert tiles == sum((N1 // 128) * (N2 // 128) for _, N1, N2, _ in shapes)
    dtab = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8).to(DEV)
    call("es_gemm_tn_grouped", ptr(dtab), len(shapes), tiles, S())
    torch.cuda.synchronize()
    for out, bias, ref, bref in refs:
        torch.testing.assert_close(out, ref, rtol=0, atol=0)
        if bias is not None:
            torch.testing.assert_close(bias, bref, rtol=0, atol=0)
    bad = (_TNProblem * 1)()
    bad[0].dy, bad[0].x, bad[0].out, bad[0].M, bad[0].N1, bad[0].N2, bad[0].ld1, bad[0].ld2 = 1, 1, 1, 10, 100, 128, 100, 128
    assert lib.es_gemm_tn_grouped_prepare(ctypes.byref(bad), 1) == -1  # N1 % 128


def _big_grouped(problems, target, timed=False):
    """es_gemm_tn_big_grouped over [(A1, A2, out, bias, M, N1, N2, ld1, ld2)] -> dims; `timed`: the
    es_gemm_tn_big_grouped_timed form (kernel-stamped events; the span must be positive)."""
    import ctypes
    from endossl.vit import _TNProblem
    lib = _lib.load()
    tab = (_TNProblem * len(problems))()
    for e, (A1, A2, out, bias, M, N1, N2, ld1, ld2) in zip(tab, problems):
        e.dy, e.x, e.out, e.bias_out = ptr(A1), ptr(A2), ptr(out), ptr(bias) if bias is not None else None
        e.M, e.N1, e.N2, e.ld1, e.ld2 = M, N1, N2, ld1, ld2
    need = lib.es_gemm_tn_big_grouped_workspace(ctypes.byref(tab), len(problems), target)
    ws = torch.empty(max(need, 1), device=DEV)
    raw = ctypes.create_string_buffer(lib.es_gemm_tn_big_grouped_table_bytes(len(problems)))
    dims = (ctypes.c_int * 3)()
    assert lib.es_gemm_tn_big_grouped_prepare(ctypes.byref(tab), len(problems), target, ptr(ws), need, raw, dims) == 0
    if need > 0:  # workspace bound enforced (one split per problem: written in place, no workspace)
        assert lib.es_gemm_tn_big_grouped_prepare(ctypes.byref(tab), len(problems), target, ptr(ws), need - 1, raw,
                                                  dims) != 0
    assert lib.es_gemm_tn_big_grouped_prepare(ctypes.byref(tab), len(problems), target, ptr(ws), need, raw, dims) == 0
    if timed:
        e0, e1 = _lib.KernelEvent(), _lib.KernelEvent()
        call("es_gemm_tn_big_grouped_timed", raw, len(problems), dims, e0.handle, e1.handle, S())
        assert e0.elapsed_time(e1) > 0.0
    else:
        call("es_gemm_tn_big_grouped", raw, len(problems), dims, S())
    torch.cuda.synchronize()
    return list(dims), ws, raw


def test_gemm_tn_big_grouped_exact_integers():
    """es_gemm_tn_big_grouped: a ViT-S block's four weight gradients (fc2 384x1536, fc1 1536x384, proj
    384x384, qkv 1152x384 -- the last with a row stride wider than N1, as the engine's K/V slice of dqkv)
    plus a problem with a ragged token count, in one split-K launch on the 384x192 tile and one reduce
    launch: exact on integer data (every partial sum is an integer below 2^24), outputs and biases
    overwritten, at a few split counts (target workgroups)."""
    g = torch.Generator().manual_seed(12)
    shapes = [(6016, 384, 1536, None), (6016, 1536, 384, None), (6016, 384, 384, None), (6016, 768, 384, 1152),
              (1000, 384, 192, None)]
    for target in (24, 120, 256):
        probs, refs = [], []
        for M, N1, N2, ld1 in shapes:
            ld1 = ld1 or N1
            A1 = _pad_rows(_int_bf16(M, ld1, lo=-2, hi=3, gen=g))
            A2 = _pad_rows(_int_bf16(M, N2, lo=-2, hi=3, gen=g))
            out = torch.full((N1, N2), 3.0, device=DEV)
            bias = torch.full((N1,), 5.0, device=DEV) if N2 != 192 else None
            probs.append((A1, A2, out, bias, M, N1, N2, ld1, N2))
            refs.append((out, bias, A1[:M, :N1].float().t() @ A2[:M].float(), A1[:M, :N1].float().sum(0)))
        dims, _, _ = _big_grouped(probs, target, timed=target in (24, 256))  # the timed form: same results
        assert dims[0] >= 23 and dims[2] == (0 if target == 24 else 2 * len(shapes) - 1)
        for out, bias, ref, bref in refs:
            torch.testing.assert_close(out, ref, rtol=0, atol=0)
            if bias is not None:
                torch.testing.assert_close(bias, bref, rtol=0, atol=0)


def test_gemm_tn_big_grouped_matches_per_gemm_launch():
    """Random bf16 data at an F1-like token count: the grouped launch's weight gradients are
    bit-identical to es_gemm_tn_ex on the same 384x192 tile (variant 7) with the same split count
    (same per-split token ranges, same kernel body, same slab-reduction order); the bias gradients
    (reduced in another order by the per-GEMM path) within fp32 rounding, and both within 1e-5 of an
    fp32 torch reference."""
    torch.manual_seed(13)
    M = 25216
    shapes = [(384, 1536), (1536, 384), (384, 384), (1152, 384)]
    probs, singles = [], []
    for N1, N2 in shapes:
        A1 = _pad_rows(torch.randn(M, N1, device=DEV).bfloat16())
        A2 = _pad_rows(torch.randn(M, N2, device=DEV).bfloat16())
        probs.append((A1, A2, torch.empty(N1, N2, device=DEV), torch.empty(N1, device=DEV), M, N1, N2, N1, N2))
    tiles = sum((N1 // 384) * (N2 // 192) for N1, N2 in shapes)
    target = 5 * tiles
    _big_grouped(probs, target)
    lib = _lib.load()
    ws = torch.empty(lib.es_gemm_tn_workspace(1536, 1536, 8), device=DEV)
    for A1, A2, out, bias, M_, N1, N2, ld1, ld2 in probs:
        o1, b1 = torch.empty(N1, N2, device=DEV), torch.empty(N1, device=DEV)
        call("es_gemm_tn_ex", ptr(A1), N1, ptr(A2), N2, M_, N1, N2, 5, ptr(ws), ptr(o1), 0, ptr(b1), 7, S())
        torch.cuda.synchronize()
        assert torch.equal(out, o1)
        torch.testing.assert_close(bias, b1, rtol=1e-6, atol=1e-4)
        ref = A1[:M_].float().t() @ A2[:M_].float()
        assert ((out - ref).norm() / ref.norm()).item() < 1e-5
        torch.testing.assert_close(bias, A1[:M_].float().sum(0), rtol=1e-5, atol=1e-2)


def test_colsum():
    torch.manual_seed(2)
    M, N = 5000, 1152
    Y = torch.randn(M, N, device=DEV).bfloat16()
    ws = torch.empty(512 * 1536, device=DEV)
    out = torch.zeros(N, device=DEV)
    call("es_colsum", ptr(Y), N, M, N, ptr(ws), 512, ptr(out), 0, S())
    torch.testing.assert_close(out, Y.float().sum(0), rtol=1e-4, atol=1e-3)
    for N2 in (384, 128, 1536):
        Y2 = torch.randn(3001, N2, device=DEV).bfloat16()
        out2 = torch.full((N2,), 2.0, device=DEV)
        call("es_colsum", ptr(Y2), N2, 3001, N2, ptr(ws), 512, ptr(out2), 1, S())
        torch.testing.assert_close(out2, Y2.float().sum(0) + 2.0, rtol=1e-4, atol=1e-3)


# ------------------------------------------------------------------------------------- attention
def _attn_ref(qkv, n, T, H):
    D = H * 64
    q, k, v = qkv.float().view(n, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-2, -1)) * 64 ** -0.5
    lse = torch.logsumexp(s, -1)
    o = (s.softmax(-1) @ v).transpose(1, 2).reshape(n * T, D)
    return o, lse


@pytest.fixture(params=[2, 3, 7], ids=["occ2", "occ3", "w7"])
def attn_occ(request):
    old = _lib.load().es_set_attn_variant(request.param)
    yield request.param
    _lib.load().es_set_attn_variant(old)


@pytest.mark.parametrize("n,T,H", [(3, 197, 6), (5, 17, 2), (2, 64, 1), (2, 250, 2), (3, 40, 2), (2, 1, 1),
                                   (2, 577, 3), (1, 300, 1)])
def test_attention_fwd(n, T, H, attn_occ):
    torch.manual_seed(T)
    D = H * 64
    qkv = _pad_rows(torch.randn(n * T, 3 * D, device=DEV).bfloat16())
    o = torch.zeros(qkv.shape[0], D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(n * H * T, device=DEV)
    call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 64 ** -0.5, S())
    o_ref, lse_ref = _attn_ref(qkv[:n * T], n, T, H)
    torch.testing.assert_close(o[:n * T].float(), o_ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse.view(n, H, T), lse_ref, rtol=1e-3, atol=2e-3)
    assert torch.all(o[n * T:] == 0)


@pytest.mark.parametrize("n,T,H", [(3, 197, 6), (4, 200, 2), (64, 197, 6)])
def test_attention_fwd_seven_waves_bit_identical(n, T, H):
    """The seven-wave forward (es_set_attn_variant 7, the default at 13 key tiles) runs each query tile's
    MFMAs, softmax and output staging exactly as the four-wave kernel (2): o and lse bit-identical, rows
    past n*T untouched."""
    D = H * 64
    torch.manual_seed(11 + T)
    qkv = _pad_rows(torch.randn(n * T, 3 * D, device=DEV).bfloat16())
    lib = _lib.load()
    res = {}
    for v in (2, 7):
        old = lib.es_set_attn_variant(v)
        o = torch.full((qkv.shape[0], D), 5.0, dtype=torch.bfloat16, device=DEV)
        lse = torch.zeros(n * H * T, device=DEV)
        call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 64 ** -0.5, S())
        torch.cuda.synchronize()
        lib.es_set_attn_variant(old)
        res[v] = (o, lse)
    assert torch.equal(res[2][0], res[7][0])
    assert torch.equal(res[2][1], res[7][1])
    assert torch.all(res[7][0][n * T:] == 5.0)


@pytest.mark.parametrize("n,T,H", [(3, 197, 6), (4, 17, 2), (3, 40, 2), (2, 250, 1), (2, 1, 1), (2, 577, 3),
                                   (1, 300, 1)])
def test_attention_bwd(n, T, H):
    torch.manual_seed(100 + T)
    D = H * 64
    qkv = _pad_rows(torch.randn(n * T, 3 * D, device=DEV).bfloat16())
    dout = _pad_rows(torch.randn(n * T, D, device=DEV).bfloat16())
    o = torch.zeros(qkv.shape[0], D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(n * H * T, device=DEV)
    call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 64 ** -0.5, S())
    dqkv = torch.zeros_like(qkv)
    delta = torch.zeros(n * H * T, device=DEV)
    call("es_attn_bwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), ptr(delta), ptr(dout), D, ptr(dqkv), 3 * D, n, T, H,
         64 ** -0.5, S())
    x = qkv[:n * T].float().requires_grad_(True)
    o_ref, _ = _attn_ref(x, n, T, H)
    o_ref.backward(dout[:n * T].float())
    ref = x.grad
    got = dqkv[:n * T].float()
    for part in range(3):
        a, b = got[:, part * D:(part + 1) * D], ref[:, part * D:(part + 1) * D]
        # scale floor: with one token O = V, so dQ = dK = 0 exactly and only an absolute bound applies
        err = (a - b).abs().max().item() / max(b.abs().max().item(), 1e-2)
        assert err < 3e-2, (part, err)
    assert torch.all(dqkv[n * T:] == 0)


@pytest.mark.parametrize("n,T,H", [(3, 197, 6), (64, 197, 6), (160, 197, 6), (3, 208, 2), (5, 193, 1), (3, 577, 12),
                                   (2, 300, 2)])
def test_attention_bwd_pipelined_matches_plain(n, T, H):
    """The software-pipelined dQ / dK-dV loops (es_set_attn_bwd_variant 1), the two-key-tiles-per-wave
    dK / dV (2), two-query-tiles dQ (3) and the single-pass kernel (4, 13 tiles: 192 < T <= 208; persistent,
    so 960 heads run several per workgroup) issue the same MFMAs on the same operands in the same order per
    tile as the plain loops (0): dqkv bit-identical (and delta, which the single pass keeps on chip), at
    T = 197 and in the 37-tile kernels (T = 577, and T = 300 with masked rows)."""
    D = H * 64
    torch.manual_seed(7 + n)
    qkv = _pad_rows(torch.randn(n * T, 3 * D, device=DEV).bfloat16())
    dout = _pad_rows(torch.randn(n * T, D, device=DEV).bfloat16())
    o = torch.zeros(qkv.shape[0], D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(n * H * T, device=DEV)
    call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 64 ** -0.5, S())
    res = {}
    lib = _lib.load()
    for v in (0, 1, 2, 3, 4):
        old = lib.es_set_attn_bwd_variant(v)
        dqkv = torch.full_like(qkv, 3.0)
        delta = torch.zeros(n * H * T, device=DEV)
        call("es_attn_bwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), ptr(delta), ptr(dout), D, ptr(dqkv), 3 * D, n, T, H,
             64 ** -0.5, S())
        torch.cuda.synchronize()
        lib.es_set_attn_bwd_variant(old)
        res[v] = (dqkv[:n * T].clone(), delta)
    for v in (1, 2, 3, 4):
        assert torch.equal(res[0][0], res[v][0]), v
        if v != 4 or (T + 15) // 16 != 13:
            assert torch.equal(res[0][1], res[v][1]), v


@pytest.mark.parametrize("n,T,H", [(3, 197, 6), (5, 17, 2), (2, 250, 2), (3, 40, 1), (2, 1, 1), (4, 256, 1),
                                   (2, 577, 2), (1, 300, 1)])
def test_attention_cls_fwd_bwd(n, T, H):
    """es_attn_cls_fwd / _bwd (the last block's CLS queries only) against the full-token kernels at
    the CLS rows -- same rounding points, fp32 summation order only -- and against fp32 torch; the
    backward equals es_attn_bwd fed a dout that is zero off the CLS rows, over EVERY token's dqkv."""
    torch.manual_seed(300 + T)
    D = H * 64
    qkv = _pad_rows(torch.randn(n * T, 3 * D, device=DEV).bfloat16())
    cls = torch.arange(n, device=DEV) * T
    # full kernels
    o = torch.zeros(qkv.shape[0], D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(n * H * T, device=DEV)
    call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 64 ** -0.5, S())
    # CLS kernels
    oc = torch.zeros(n, D, dtype=torch.bfloat16, device=DEV)
    lc = torch.zeros(n * H, device=DEV)
    call("es_attn_cls_fwd", ptr(qkv), 3 * D, ptr(oc), D, ptr(lc), n, T, H, 64 ** -0.5, S())
    torch.cuda.synchronize()
    torch.testing.assert_close(lc.view(n, H), lse.view(n, H, T)[:, :, 0], rtol=1e-5, atol=1e-5)
    # the bf16 outputs agree to within one rounding step of the output (past T = 256 the long kernel's
    # online softmax rounds P against the running, not the final, row max: a bound relative to the
    # row's scale)
    if T <= 256:
        assert ((oc.float() - o[cls].float()).abs() <= o[cls].float().abs() * 2 ** -7 + 1e-6).all()
    else:
        assert (oc.float() - o[cls].float()).abs().max() <= 1e-2 * o[cls].float().abs().max()
    o_ref, _ = _attn_ref(qkv[:n * T], n, T, H)
    torch.testing.assert_close(oc.float(), o_ref[cls], rtol=2e-2, atol=2e-2)
    # backward: dout nonzero on the CLS rows only
    doc = torch.randn(n, D, device=DEV).bfloat16()
    dout = torch.zeros(qkv.shape[0], D, dtype=torch.bfloat16, device=DEV)
    dout[cls] = doc
    dq_full = torch.zeros_like(qkv)
    delta = torch.zeros(n * H * T, device=DEV)
    call("es_attn_bwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), ptr(delta), ptr(dout), D, ptr(dq_full), 3 * D, n, T,
         H, 64 ** -0.5, S())
    dq_cls = torch.full_like(qkv, float("nan"))  # every token row must be written
    dq_cls[n * T:] = 0
    call("es_attn_cls_bwd", ptr(qkv), 3 * D, ptr(oc), D, ptr(lc), ptr(doc), D, ptr(dq_cls), 3 * D, n, T, H,
         64 ** -0.5, S())
    torch.cuda.synchronize()
    assert torch.isfinite(dq_cls).all()
    x = qkv[:n * T].float().requires_grad_(True)
    o_r, _ = _attn_ref(x, n, T, H)
    o_r.backward(dout[:n * T].float())
    for part in range(3):
        a = dq_cls[:n * T, part * D:(part + 1) * D].float()
        b = dq_full[:n * T, part * D:(part + 1) * D].float()
        r = x.grad[:, part * D:(part + 1) * D]
        scale = max(r.abs().max().item(), 1e-2)
        assert (a - b).abs().max().item() / scale < 1e-2, part
        assert (a - r).abs().max().item() / scale < 3e-2, part
    qpart = dq_cls[:n * T, :D].view(n, T, D)
    assert torch.all(qpart[:, 1:] == 0)


# ------------------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("D", [128, 384, 768])
@pytest.mark.parametrize("M", [1000, 1001, 7])
def test_layernorm_fwd_bwd(D, M):
    torch.manual_seed(D)
    x = torch.randn(M, D, device=DEV) * 2 + 0.5
    gamma = 1 + 0.1 * torch.randn(D, device=DEV)
    beta = 0.1 * torch.randn(D, device=DEV)
    y = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    mean, rstd = torch.zeros(M, device=DEV), torch.zeros(M, device=DEV)
    call("es_layernorm_fwd", ptr(x), D, ptr(gamma), ptr(beta), ptr(y), D, ptr(mean), ptr(rstd), M, D, 1e-6, S())
    xr = x.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (D,), gr, br, 1e-6)
    torch.testing.assert_close(y.float(), yr.detach(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(mean, x.mean(1), rtol=1e-5, atol=1e-5)
    # the one-shot forward (a workgroup per 8 rows) and the grid-stride one (few workgroups: each wave walks
    # many row pairs with the next pair's loads in flight) are bit-identical
    lib = _lib.load()
    for grid in (0, 3):
        old = lib.es_set_ln_fwd_grid(grid)
        y2 = torch.full_like(y, 7.0)
        m2, r2 = torch.zeros_like(mean), torch.zeros_like(rstd)
        call("es_layernorm_fwd", ptr(x), D, ptr(gamma), ptr(beta), ptr(y2), D, ptr(m2), ptr(r2), M, D, 1e-6, S())
        torch.cuda.synchronize()
        lib.es_set_ln_fwd_grid(old)
        assert torch.equal(y2, y) and torch.equal(m2, mean) and torch.equal(r2, rstd), grid
    dy = torch.randn(M, D, device=DEV)
    dres = torch.randn(M, D, device=DEV)
    yr.backward(dy)
    dx = torch.zeros(M, D, device=DEV)
    dxb = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    dg, db = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    ws = torch.empty(2 * 1024 * D, device=DEV)
    call("es_layernorm_bwd", ptr(dy), D, ptr(x), D, ptr(mean), ptr(rstd), ptr(gamma), ptr(dres), D, ptr(dx), D,
         ptr(dxb), D, ptr(dg), ptr(db), ptr(ws), 1024, M, D, 0, S())
    torch.testing.assert_close(dx, xr.grad + dres, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dxb.float(), (xr.grad + dres), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dg, gr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-3)
    # few workgroups: each wave walks many row pairs (grid-stride path)
    dx2, dg2, db2 = torch.zeros_like(dx), torch.zeros_like(dg), torch.zeros_like(db)
    call("es_layernorm_bwd", ptr(dy), D, ptr(x), D, ptr(mean), ptr(rstd), ptr(gamma), ptr(dres), D, ptr(dx2), D,
         None, D, ptr(dg2), ptr(db2), ptr(ws), 5, M, D, 0, S())
    torch.testing.assert_close(dx2, dx, rtol=0, atol=0)
    torch.testing.assert_close(dg2, gr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db2, br.grad, rtol=1e-4, atol=1e-3)
    # bf16 dy (es_layernorm_bwd_b16): the fp32 kernel's result on the same bf16-rounded dy, exactly
    dyb = dy.bfloat16()
    dx3, dg3, db3 = torch.zeros_like(dx), torch.zeros_like(dg), torch.zeros_like(db)
    call("es_layernorm_bwd_b16", ptr(dyb), D, ptr(x), D, ptr(mean), ptr(rstd), ptr(gamma), ptr(dres), D, ptr(dx3), D,
         None, D, ptr(dg3), ptr(db3), ptr(ws), 1024, M, D, 0, S())
    dyr = dyb.float()
    dx4, dg4, db4 = torch.zeros_like(dx), torch.zeros_like(dg), torch.zeros_like(db)
    call("es_layernorm_bwd", ptr(dyr), D, ptr(x), D, ptr(mean), ptr(rstd), ptr(gamma), ptr(dres), D, ptr(dx4), D,
         None, D, ptr(dg4), ptr(db4), ptr(ws), 1024, M, D, 0, S())
    torch.testing.assert_close(dx3, dx4, rtol=0, atol=0)
    torch.testing.assert_close(dg3, dg4, rtol=0, atol=0)
    torch.testing.assert_close(db3, db4, rtol=0, atol=0)
    # dgamma / dbeta leave through one paired reduction launch: bit-identical to es_reduce_partials over
    # the partials the kernel left in the workspace (pg = ws[:G*D], pb = ws[G*D:2*G*D]); accumulate adds
    G = min(1024, (M + 7) // 8)
    rg, rb = torch.zeros_like(dg), torch.zeros_like(db)
    call("es_reduce_partials", ptr(ws), ptr(rg), G, D, 0, S())
    call("es_reduce_partials", ptr(ws[G * D:]), ptr(rb), G, D, 0, S())
    torch.testing.assert_close(dg4, rg, rtol=0, atol=0)
    torch.testing.assert_close(db4, rb, rtol=0, atol=0)
    dg5, db5 = dg4.clone(), db4.clone()
    call("es_layernorm_bwd", ptr(dyr), D, ptr(x), D, ptr(mean), ptr(rstd), ptr(gamma), ptr(dres), D, ptr(dx4), D,
         None, D, ptr(dg5), ptr(db5), ptr(ws), 1024, M, D, 1, S())
    torch.testing.assert_close(dg5, dg4 + rg, rtol=0, atol=0)
    torch.testing.assert_close(db5, db4 + rb, rtol=0, atol=0)


# ------------------------------------------------------------------------------------- ViT ends
def test_im2col_matches_unfold():
    torch.manual_seed(3)
    n, Sz = 3, 64
    img = torch.randn(n, 3, Sz, Sz, device=DEV)
    pt = torch.zeros(n * 16, 768, dtype=torch.bfloat16, device=DEV)
    call("es_patch_im2col", ptr(img), ptr(pt), n, Sz, 16, S())
    ref = F.unfold(img, 16, stride=16).transpose(1, 2).reshape(n * 16, 768)
    torch.testing.assert_close(pt.float(), ref.bfloat16().float(), rtol=0, atol=0)


@pytest.mark.parametrize("n,Sz", [(5, 224), (3, 64), (2, 384), (448, 224)])
def test_im2col_u8_matches_normalised_fp32(n, Sz):
    """es_patch_im2col_u8 (uint8 pixels, ToTensor + Normalize fused into the gather) == es_patch_im2col over
    the same pixels normalised in fp32, bit for bit, incl. the F1 weak batch (448 images) and the ViT-B/16
    384^2 size."""
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    g = torch.Generator().manual_seed(n + Sz)
    u8 = torch.randint(0, 256, (n, 3, Sz, Sz), generator=g, dtype=torch.uint8)
    f32 = ((u8.float() / 255.0 - torch.tensor(mean).view(1, 3, 1, 1)) / torch.tensor(std).view(1, 3, 1, 1)).to(DEV)
    rows = n * (Sz // 16) ** 2
    pa = torch.full((rows + 7, 768), 9.0, dtype=torch.bfloat16, device=DEV)
    pb = torch.zeros(rows, 768, dtype=torch.bfloat16, device=DEV)
    call("es_patch_im2col_u8", ptr(u8.to(DEV)), *mean, *std, ptr(pa), n, Sz, 16, S())
    call("es_patch_im2col", ptr(f32), ptr(pb), n, Sz, 16, S())
    torch.cuda.synchronize()
    assert torch.equal(pa[:rows], pb)
    assert torch.all(pa[rows:] == 9.0)
    if n == 5:  # pixels 8-B but not 16-B aligned: the element-wise gather instead of the LDS band kernel
        buf = torch.zeros(u8.numel() + 16, dtype=torch.uint8, device=DEV)
        buf[8:8 + u8.numel()] = u8.reshape(-1).to(DEV)
        pc = torch.full((rows, 768), 9.0, dtype=torch.bfloat16, device=DEV)
        call("es_patch_im2col_u8", ptr(buf) + 8, *mean, *std, ptr(pc), n, Sz, 16, S())
        torch.cuda.synchronize()
        assert torch.equal(pc, pb)


@pytest.mark.parametrize("n", [37, 512])
def test_cls_head_fwd_bwd(n):
    torch.manual_seed(4)
    T, D, C = 5, 384, 23
    x = torch.randn(n * T, D, device=DEV)
    gamma = 1 + 0.1 * torch.randn(D, device=DEV)
    beta = 0.1 * torch.randn(D, device=DEV)
    W = 0.05 * torch.randn(C, D, device=DEV)
    b = 0.1 * torch.randn(C, device=DEV)
    logits = torch.zeros(n, C, device=DEV)
    xhat, rstd = torch.zeros(n, D, device=DEV), torch.zeros(n, device=DEV)
    call("es_cls_head_fwd", ptr(x), D, T, ptr(gamma), ptr(beta), ptr(W), ptr(b), ptr(logits), C, ptr(xhat), ptr(rstd),
         n, D, C, 1e-6, S())
    xr, gr, br, Wr, bhr = (t.clone().requires_grad_(True) for t in (x, gamma, beta, W, b))
    lr = F.linear(F.layer_norm(xr.view(n, T, D)[:, 0], (D,), gr, br, 1e-6), Wr, bhr)
    torch.testing.assert_close(logits, lr.detach(), rtol=1e-5, atol=1e-5)
    dl = torch.randn(n, C, device=DEV)
    lr.backward(dl)
    dx = torch.zeros(n * T, D, device=DEV)
    dyn = torch.zeros(n, D, device=DEV)
    dW, db, dg, dbt = torch.zeros_like(W), torch.zeros_like(b), torch.zeros_like(gamma), torch.zeros_like(beta)
    call("es_cls_head_bwd", ptr(dl), C, ptr(W), ptr(gamma), ptr(beta), ptr(xhat), ptr(rstd), ptr(dyn), ptr(dx), D, T,
         ptr(dW), ptr(db), ptr(dg), ptr(dbt), n, D, C, S())
    torch.testing.assert_close(dx, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dW, Wr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(db, bhr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dg, gr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dbt, br.grad, rtol=1e-4, atol=1e-5)
    # the parameter sums run in a fixed order (no atomics): a second launch accumulating onto a copy of the
    # first result gives exactly twice each sum's bits added -- i.e. a repeat from zero is bit-identical
    dW2, db2, dg2, dbt2 = torch.zeros_like(W), torch.zeros_like(b), torch.zeros_like(gamma), torch.zeros_like(beta)
    call("es_cls_head_bwd", ptr(dl), C, ptr(W), ptr(gamma), ptr(beta), ptr(xhat), ptr(rstd), ptr(dyn), ptr(dx), D, T,
         ptr(dW2), ptr(db2), ptr(dg2), ptr(dbt2), n, D, C, S())
    torch.cuda.synchronize()
    for a, c in ((dW, dW2), (db, db2), (dg, dg2), (dbt, dbt2)):
        assert torch.equal(a, c)
    call("es_cls_head_bwd", ptr(dl), C, ptr(W), ptr(gamma), ptr(beta), ptr(xhat), ptr(rstd), ptr(dyn), ptr(dx), D, T,
         ptr(dW2), ptr(db2), ptr(dg2), ptr(dbt2), n, D, C, S())  # accumulates (+=), like the atomics did
    torch.testing.assert_close(dW2, 2 * dW, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(db2, 2 * db, rtol=1e-6, atol=1e-7)
    # es_cls_head_bwd_ex(accumulate = 0) writes the sums over whatever the buffers held (NaN here): the bits of
    # the accumulate-onto-zero form
    nanf = lambda t: torch.full_like(t, float("nan"))  # noqa: E731
    dW3, db3, dg3, dbt3 = nanf(W), nanf(b), nanf(gamma), nanf(beta)
    call("es_cls_head_bwd_ex", ptr(dl), C, ptr(W), ptr(gamma), ptr(beta), ptr(xhat), ptr(rstd), ptr(dyn), ptr(dx), D,
         T, ptr(dW3), ptr(db3), ptr(dg3), ptr(dbt3), n, D, C, 0, S())
    torch.cuda.synchronize()
    for a, c in ((dW, dW3), (db, db3), (dg, dg3), (dbt, dbt3)):
        assert torch.equal(a, c)


def test_embed_bwd():
    torch.manual_seed(5)
    n, T, D = 6, 17, 128
    dx = torch.randn(n * T, D, device=DEV)
    dp = torch.zeros(n * (T - 1), D, dtype=torch.bfloat16, device=DEV)
    dpos, dcls = torch.zeros(T, D, device=DEV), torch.zeros(D, device=DEV)
    call("es_embed_bwd", ptr(dx), D, ptr(dp), D, ptr(dpos), ptr(dcls), n, T, D, 0, S())
    v = dx.view(n, T, D)
    torch.testing.assert_close(dpos, v.sum(0), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dcls, v[:, 0].sum(0), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dp.float(), v[:, 1:].reshape(-1, D).bfloat16().float(), rtol=0, atol=0)
    # the four-features-per-lane kernel (above: D, strides multiples of 4) vs the per-feature one (a row stride of
    # D + 1 selects it): the same sums in the same order, bit for bit; accumulate adds onto the outputs
    dxp = torch.zeros(n * T, D + 1, device=DEV)
    dxp[:, :D] = dx
    dp2 = torch.zeros_like(dp)
    dpos2, dcls2 = torch.zeros_like(dpos), torch.zeros_like(dcls)
    call("es_embed_bwd", ptr(dxp), D + 1, ptr(dp2), D, ptr(dpos2), ptr(dcls2), n, T, D, 0, S())
    torch.cuda.synchronize()
    assert torch.equal(dp2, dp) and torch.equal(dpos2, dpos) and torch.equal(dcls2, dcls)
    call("es_embed_bwd", ptr(dx), D, ptr(dp), D, ptr(dpos), ptr(dcls), n, T, D, 1, S())
    torch.testing.assert_close(dpos, 2 * dpos2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(dcls, 2 * dcls2, rtol=1e-6, atol=1e-6)


# ------------------------------------------------------------------------------------- losses (golden)
def test_consistency_kernel_vs_reference_fixture(golden):
    for tag in ("0p7", "0p95", "median"):
        d = golden(f"consistency_{tag}.npz")
        lw = torch.tensor(d["logits_w"], device=DEV)
        ls = torch.tensor(d["logits_s"], device=DEV)
        n, C = ls.shape
        tau = float(d["tau"])
        pl = torch.zeros(n, dtype=torch.int32, device=DEV)
        mask = torch.zeros(n, dtype=torch.uint8, device=DEV)
        rows = torch.zeros(n, device=DEV)
        dls = torch.zeros(n, C, device=DEV)
        out = torch.zeros(2, device=DEV)
        call("es_fm_consistency_fwd_bwd", ptr(lw), C, ptr(ls), C, n, C, tau, 1.0 / n, ptr(pl), ptr(mask), ptr(rows),
             ptr(dls), C, ptr(out), S())
        torch.cuda.synchronize()
        pmax = torch.softmax(torch.tensor(d["logits_w"], dtype=torch.float64), -1).max(-1).values.numpy()
        near = np.abs(pmax - tau) < 1e-6  # rows whose max-prob is within ulps of tau: mask undefined
        np.testing.assert_array_equal(pl.cpu().numpy(), d["pseudo_label"])  # integer labels bit-exact
        np.testing.assert_array_equal(mask.cpu().numpy()[~near], d["mask"][~near].astype(np.uint8))
        # the fixture's ce_rows are the reference's per-row CE BEFORE `* mask` (code/loss.py:157-160)
        rows_h = rows.cpu().numpy()
        np.testing.assert_allclose(rows_h[~near], (d["ce_rows"] * d["mask"])[~near], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(out[0].item(), rows_h.mean(), rtol=1e-5)
        slack = d["ce_rows"][near].sum() / n  # a row exactly at tau may flip: its whole CE moves the mean
        assert abs(out[0].item() - float(d["loss"])) <= 1e-5 * float(d["loss"]) + slack
        np.testing.assert_allclose(out[1].item(), float(d["mask_mean"]), rtol=0, atol=1.0 / n * near.sum() + 1e-7)
        ok = ~near
        np.testing.assert_allclose(dls.cpu().numpy()[ok], d["grad_logits_s"][ok], rtol=1e-4, atol=1e-7)


def test_poly_kernel_vs_reference_fixture(golden):
    for tag in ("weighted", "plain"):
        d = golden(f"poly_{tag}.npz")
        lg = torch.tensor(d["logits"], device=DEV)
        y = torch.tensor(d["targets"], device=DEV)
        w = torch.tensor(d["weights"], device=DEV) if d["weights"].size else None
        n, C = lg.shape
        dl = torch.zeros(n, C, device=DEV)
        out = torch.zeros(1, device=DEV)
        call("es_poly_ce_fwd_bwd", ptr(lg), C, ptr(y), ptr(w), n, C, 2.0, 1.0 / n, ptr(dl), C, ptr(out), S())
        np.testing.assert_allclose(out.item(), float(d["loss"]), rtol=1e-5)
        np.testing.assert_allclose(dl.cpu().numpy(), d["grad_logits"], rtol=1e-4, atol=1e-6)


def test_loss_module_api_autograd(golden):
    from endossl.loss import ce_loss, consistency_loss
    d = golden("consistency_0p95.npz")
    lw = torch.tensor(d["logits_w"], device=DEV)
    ls = torch.tensor(d["logits_s"], device=DEV).requires_grad_(True)
    loss, mm = consistency_loss(lw, ls, T=1.0, p_cutoff=float(d["tau"]))
    (2.0 * loss).backward()
    np.testing.assert_allclose(ls.grad.cpu().numpy(), 2.0 * d["grad_logits_s"], rtol=1e-4, atol=1e-7)
    d = golden("poly_weighted.npz")
    x = torch.tensor(d["logits"], device=DEV).requires_grad_(True)
    lx = ce_loss(x, torch.tensor(d["targets"], device=DEV), class_weights=torch.tensor(d["weights"], device=DEV),
                 reduction="mean", type_loss="poly")
    lx.backward()
    np.testing.assert_allclose(lx.item(), float(d["loss"]), rtol=1e-5)
    np.testing.assert_allclose(x.grad.cpu().numpy(), d["grad_logits"], rtol=1e-4, atol=1e-6)


# ------------------------------------------------------------------------------------- EMA / Adam
def test_ema_multi_bit_exact_vs_reference_fixture(golden):
    import torch.nn as nn
    from endossl.ema import ModelEMA
    d = golden("ema.npz")
    keys = [k.split("/", 1)[1] for k in d.files if k.startswith("ema_before/")]
    m = nn.Sequential(nn.Linear(16, 32), nn.BatchNorm1d(32), nn.ReLU(), nn.Linear(32, 5)).to(DEV)
    m.load_state_dict({k: torch.tensor(d["ema_before/" + k]) for k in keys})
    e = ModelEMA(m, decay=0.999, device=DEV)
    m.load_state_dict({k: torch.tensor(d["model/" + k]) for k in keys})
    e.update(m)
    torch.cuda.synchronize()
    for k, v in e.ema.state_dict().items():
        np.testing.assert_array_equal(v.cpu().numpy(), d["ema_after/" + k], err_msg=k)


def test_adam_ema_step_vs_torch_adam():
    torch.manual_seed(6)
    n = 10_000
    p0 = torch.randn(n)
    grads = [torch.randn(n) * 10 ** (-i) for i in range(3)]
    # torch.optim.Adam on CPU = the reference optimizer
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0)
    er = p0.clone()
    p, m, v, e = p0.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV), p0.to(DEV)
    for t, gr in enumerate(grads, 1):
        pr.grad = gr.clone()
        opt.step()
        er = 0.999 * er + (1.0 - 0.999) * pr.detach()
        g = gr.to(DEV)
        bc1, bc2 = 1 - 0.9 ** t, 1 - 0.999 ** t
        call("es_adam_ema_step", ptr(p), ptr(g), ptr(m), ptr(v), ptr(e), n, 0.9, 0.999, 1e-8, -1e-3 / bc1,
             math.sqrt(bc2), 0.999, 1.0 - 0.999, 1.0, S())
    torch.testing.assert_close(p.cpu(), pr.detach(), rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(e.cpu(), er, rtol=1e-6, atol=1e-7)


def test_pack_weights_exact():
    from endossl.vit import Engine, NativeViT, ViTConfig
    m = NativeViT(ViTConfig(img_size=64, dim=128, depth=2, heads=2), seed=3).to(DEV)
    eng = m.engine()
    eng.pack(m.flat)
    torch.cuda.synchronize()
    sd = m.state_dict()
    for name, wb in eng.wb.items():
        W = sd[name].reshape(wb.shape[0], -1)
        assert torch.equal(wb, W.bfloat16()), name
        if name in eng.wt:
            assert torch.equal(eng.wt[name], W.t().contiguous().bfloat16()), name


def test_conv_pack_multi_matches_single_pack():
    """es_conv2d_pack_bf16_multi (every conv weight of a model in one launch) writes the same images as
    es_conv2d_pack_bf16 per weight: wp [Cout][k k][Cin], wt [Cin][k k][Cout], bit for bit."""
    import ctypes
    from endossl import _lib
    shapes = [(64, 32, 3), (256, 64, 1), (32, 96, 7), (768, 256, 1), (128, 128, 3), (512, 512, 3), (100, 60, 3)]
    g = torch.Generator().manual_seed(5)
    ws = [torch.randn(co, ci, k, k, generator=g).to(DEV) for co, ci, k in shapes]
    outs = [(torch.empty(w.numel(), dtype=torch.bfloat16, device=DEV),
             torch.empty(w.numel(), dtype=torch.bfloat16, device=DEV)) for w in ws]
    esz = _lib.load().es_conv_pack_entry_size()
    raw = bytearray(esz * len(ws))
    for j, ((co, ci, k), w, (wp, wt)) in enumerate(zip(shapes, ws, outs)):
        ent = (ctypes.c_void_p(ptr(w)), ctypes.c_void_p(ptr(wp)), ctypes.c_void_p(ptr(wt)), ctypes.c_int(co),
               ctypes.c_int(ci), ctypes.c_int(k * k), ctypes.c_int(0))
        buf = b"".join(bytes(e) for e in ent)
        raw[j * esz:j * esz + len(buf)] = buf
    tab = torch.frombuffer(raw, dtype=torch.uint8).to(DEV)
    call("es_conv2d_pack_bf16_multi", ptr(tab), len(ws), max(w.numel() for w in ws), S())
    for (co, ci, k), w, (wp, wt) in zip(shapes, ws, outs):
        rp = torch.empty_like(wp)
        rt = torch.empty_like(wt)
        call("es_conv2d_pack_bf16", ptr(w), co, ci, k, k, ptr(rp), ptr(rt), S())
        torch.cuda.synchronize()
        assert torch.equal(wp, rp) and torch.equal(wt, rt), (co, ci, k)
        assert torch.equal(wp.view(co, k * k, ci), w.permute(0, 2, 3, 1).reshape(co, k * k, ci).bfloat16())
        assert torch.equal(wt.view(ci, k * k, co), w.permute(1, 2, 3, 0).reshape(ci, k * k, co).bfloat16())


def test_conformer_conv_pack_multi_after_first_version():
    """NativeConformer.conv_pack: the first parameter version packs per weight and records the table; the
    next version packs every recorded weight in one launch; the images equal a fresh per-weight pack."""
    from endossl.conformer import ConformerConfig, NativeConformer
    m = NativeConformer(ConformerConfig(img_size=64, base_channel=32, embed_dim=128, depth=3, heads=2), seed=1).to(DEV)
    x = torch.randn(2, 3, 64, 64, device=DEV)
    m.train()
    m(x)
    assert m._cpack and m._cpack_tab is None and m._cpack_next
    with torch.no_grad():
        m.flat.add_(0.01 * torch.randn_like(m.flat))
    m.mark_updated()
    m(x)
    torch.cuda.synchronize()
    assert m._cpack_tab is not None and m._cpack_tab[1] == len(m._cpack)
    for name, (ver, wp, wt, (co, ci, k)) in m._cpack.items():
        assert ver == m.version, name
        rp, rt = torch.empty_like(wp), torch.empty_like(wt)
        call("es_conv2d_pack_bf16", ptr(m.pview(name)), co, ci, k, k, ptr(rp), ptr(rt), S())
        torch.cuda.synchronize()
        assert torch.equal(wp, rp) and torch.equal(wt, rt), name


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,p", [(3, 12, 64, 128, 3, 1, 1), (2, 16, 128, 64, 1, 1, 0),
                                                (2, 15, 64, 256, 3, 2, 1), (3, 9, 32, 96, 1, 2, 0),
                                                (2, 24, 64, 768, 4, 4, 0), (1, 7, 96, 128, 3, 1, 1),
                                                (2, 13, 128, 128, 3, 2, 1), (2, 10, 256, 64, 3, 1, 1),
                                                (3, 11, 96, 32, 3, 1, 1)])
def test_conv_ring_bit_identical(N, H, Cin, Cout, k, s, p):
    """The bf16-map forward (plain and with BatchNorm statistics) and data-gradient convs on the LDS-DMA ring kernel
    (es_set_conv_ring 3 / 4) and on the staged kernel's branch-free gathers (es_set_conv_dw_buf 1) against the
    staged kernel's branchy gathers (ring 0, dw_buf 0): outputs, accumulated outputs
    and statistics partials BIT-identical -- padding, strides / stride phases, pixel counts off the 128-pixel tile,
    64- and 128-column tiles, bf16 and fp32 outputs (the widening forwards stay on the staged kernel either way:
    Cin >= Cout cases exercise the ring forward)."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(N * 100 + H)
    Ho = (H + 2 * p - k) // s + 1
    M = N * Ho * Ho
    x = torch.randn(N, H, H, Cin, device=DEV, generator=g).bfloat16()
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) * 0.05
    dy = torch.randn(N, Ho, Ho, Cout, device=DEV, generator=g).bfloat16()
    wp = torch.empty(w.numel(), dtype=torch.bfloat16, device=DEV)
    wt = torch.empty_like(wp)
    call("es_conv2d_pack_bf16", ptr(w), Cout, Cin, k, k, ptr(wp), ptr(wt), S())
    bias = torch.randn(Cout, device=DEV, generator=g)
    xs = (H * H * Cin, H * Cin, Cin, 1)
    ys = (Ho * Ho * Cout, Ho * Cout, Cout)
    res = {}
    try:
        for ring, dwb in ((0, 0), (0, 1), (3, 1), (4, 1)):  # (0, 0): the staged kernel with its branchy gathers
            assert lib.es_set_conv_ring(ring) in (0, 3, 4)
            assert lib.es_set_conv_dw_buf(dwb) in (0, 1)
            out = {}
            for od, fl in ((torch.bfloat16, 3), (torch.float32, 1)):
                y = torch.zeros(N, Ho, Ho, Cout, device=DEV, dtype=od)
                part = torch.zeros(lib.es_conv2d_bnstats_size(M, Cout), device=DEV)
                call("es_conv2d_fwd_bf16_ex", ptr(x), N, H, H, Cin, *xs, ptr(wp), ptr(bias), Cout, k, k, s, p, ptr(y), *ys,
                     0, ptr(part), fl, S())
                ya = torch.randn(N, Ho, Ho, Cout, device=DEV, generator=torch.Generator(device=DEV).manual_seed(7)).to(od)
                call("es_conv2d_fwd_bf16_ex", ptr(x), N, H, H, Cin, *xs, ptr(wp), None, Cout, k, k, s, p, ptr(ya), *ys,
                     1, None, fl, S())
                dx = torch.zeros(N, H, H, Cin, device=DEV, dtype=od)
                call("es_conv2d_bwd_data_bf16_ex", ptr(dy), *ys, ptr(wt), N, H, H, Cin, Cout, k, k, s, p, ptr(dx), *xs, 0,
                     fl, S())
                torch.cuda.synchronize()
                out[od] = (y, part, ya, dx)
            res[(ring, dwb)] = out
    finally:
        lib.es_set_conv_ring(3)
        lib.es_set_conv_dw_buf(1)
    for key in ((0, 1), (3, 1), (4, 1)):
        for od in (torch.bfloat16, torch.float32):
            for name, a, b in zip(("y", "stats", "y_acc", "dx"), res[key][od], res[(0, 0)][od]):
                assert torch.equal(a, b), (key, od, name, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,p", [(16, 7, 512, 512, 3, 1, 1), (16, 14, 256, 512, 3, 2, 1),
                                                (16, 14, 256, 512, 1, 2, 0), (16, 14, 256, 256, 3, 1, 1),
                                                (3, 12, 128, 128, 3, 1, 1)])
def test_conv_small_grid_tile_bit_identical(N, H, Cin, Cout, k, s, p):
    """es_set_conv_small: a bf16 conv forward (plain, with BatchNorm statistics, accumulating) and data gradient
    whose 128-channel tiling launches few workgroups (P0's layer-3 / layer-4 shapes at B = 16) on the 64-channel
    tile, against the 128-channel tile: every output and statistics partial BIT-identical."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(N * 31 + H)
    Ho = (H + 2 * p - k) // s + 1
    M = N * Ho * Ho
    x = torch.randn(N, H, H, Cin, device=DEV, generator=g).bfloat16()
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) * 0.05
    dy = torch.randn(N, Ho, Ho, Cout, device=DEV, generator=g).bfloat16()
    wp = torch.empty(w.numel(), dtype=torch.bfloat16, device=DEV)
    wt = torch.empty_like(wp)
    call("es_conv2d_pack_bf16", ptr(w), Cout, Cin, k, k, ptr(wp), ptr(wt), S())
    bias = torch.randn(Cout, device=DEV, generator=g)
    xs = (H * H * Cin, H * Cin, Cin, 1)
    ys = (Ho * Ho * Cout, Ho * Cout, Cout)
    res = {}
    try:
        for small in (0, 1 << 20):  # 0: always the 128-channel tile; huge: the 64-channel tile wherever it applies
            assert lib.es_set_conv_small(small) >= 0
            out = []
            for od, fl in ((torch.bfloat16, 3), (torch.float32, 1)):
                y = torch.zeros(N, Ho, Ho, Cout, device=DEV, dtype=od)
                part = torch.zeros(lib.es_conv2d_bnstats_size(M, Cout), device=DEV)
                call("es_conv2d_fwd_bf16_ex", ptr(x), N, H, H, Cin, *xs, ptr(wp), ptr(bias), Cout, k, k, s, p, ptr(y), *ys,
                     0, ptr(part), fl, S())
                ya = torch.randn(N, Ho, Ho, Cout, device=DEV, generator=torch.Generator(device=DEV).manual_seed(7)).to(od)
                call("es_conv2d_fwd_bf16_ex", ptr(x), N, H, H, Cin, *xs, ptr(wp), None, Cout, k, k, s, p, ptr(ya), *ys,
                     1, None, fl, S())
                dx = torch.zeros(N, H, H, Cin, device=DEV, dtype=od)
                call("es_conv2d_bwd_data_bf16_ex", ptr(dy), *ys, ptr(wt), N, H, H, Cin, Cout, k, k, s, p, ptr(dx), *xs, 0,
                     fl, S())
                torch.cuda.synchronize()
                out += [y, part, ya, dx]
            res[small] = out
    finally:
        lib.es_set_conv_small(128)
    for i, (a, b) in enumerate(zip(res[1 << 20], res[0])):
        assert torch.equal(a, b), (i, (a.float() - b.float()).abs().max().item())


@pytest.mark.parametrize("N,H,Cin,Cout,k,s,p", [(3, 12, 64, 128, 3, 1, 1), (2, 16, 128, 64, 1, 1, 0),
                                                (2, 15, 64, 256, 3, 2, 1), (3, 9, 32, 96, 1, 2, 0),
                                                (2, 24, 64, 768, 4, 4, 0), (2, 40, 64, 64, 3, 1, 1),
                                                (1, 4, 64, 64, 3, 1, 1)])
def test_conv_dw_branch_free_bit_identical(N, H, Cin, Cout, k, s, p):
    """The bf16 conv weight gradient with branch-free loads / pixel walk (es_set_conv_dw_buf 1) against the branchy
    kernel (0): the weight gradient BIT-identical, plain and with the input BatchNorm applied by the gather, bf16 and
    fp32 dy; maps wide and narrow (Wo < 32: several rows per 32-pixel step; a 2 x 2 map takes the branchy kernel)."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(N * 10 + H)
    Ho = (H + 2 * p - k) // s + 1
    M = N * Ho * Ho
    x = torch.randn(N, H, H, Cin, device=DEV, generator=g).bfloat16()
    mean, rstd = torch.randn(Cin, device=DEV, generator=g) * 0.1, torch.rand(Cin, device=DEV, generator=g) + 0.5
    gam, bet = torch.rand(Cin, device=DEV, generator=g) + 0.5, torch.randn(Cin, device=DEV, generator=g) * 0.1
    xs = (H * H * Cin, H * Cin, Cin, 1)
    ys = (Ho * Ho * Cout, Ho * Cout, Cout)
    ws = torch.empty(lib.es_conv2d_bwd_weight_bf16_workspace(M, Cout, Cin, k, k, 0), device=DEV)
    res = {}
    try:
        for buf in (0, 1):
            lib.es_set_conv_dw_buf(buf)
            out = []
            for dyt, fl in ((torch.bfloat16, 3), (torch.float32, 1)):
                dy = torch.randn(N, Ho, Ho, Cout, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3)).to(dyt)
                dw = torch.zeros(Cout, Cin, k, k, device=DEV)
                call("es_conv2d_bwd_weight_bf16_ex", ptr(x), N, H, H, Cin, *xs, ptr(dy), *ys, Cout, k, k, s, p, 0,
                     ptr(ws), ptr(dw), 0, fl, S())
                dwb = torch.zeros_like(dw)
                call("es_conv2d_bwd_weight_bf16_bnin_ex", ptr(x), N, H, H, Cin, *xs, ptr(dy), *ys, Cout, k, k, s, p, 0,
                     ptr(ws), ptr(dwb), 0, fl, ptr(mean), ptr(rstd), ptr(gam), ptr(bet), S())
                torch.cuda.synchronize()
                out += [dw, dwb]
            res[buf] = out
    finally:
        lib.es_set_conv_dw_buf(1)
    for a, b in zip(res[1], res[0]):
        assert b.abs().max() > 0
        assert torch.equal(a, b), (a - b).abs().max().item()
