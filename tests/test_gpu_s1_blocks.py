"""Teacher-forced per-op parity of the S1 transformer branch at its own shape (BASELINE configs[4]).

One SemiFormer step (code/semiformer.py:103-146) on Conformer-B at 384^2 (code/models/conformer.py:306-310:
embed 768, depth 12, 12 heads, 577 tokens), B=1, mu=7 (15 images: M = 8,655 token rows per GEMM).  The
conformer module's block hook (conformer.BLOCK_CAPTURE) hands over, for each of the 12 transformer blocks
(`Block`, code/models/conformer.py:27-72), the operands and outputs of every kernel the block launched --
LN1, the qkv GEMM (the 256 x 256 tile at D = 768), the long-sequence attention forward (attn_fwd_long, 37
key tiles), proj GEMM + residual, LN2, fc1 GEMM + GELU (pre-activation and activation), fc2 GEMM + residual;
in reverse bf16(dY), fc2 data gradient x GELU'(pre), fc1 data gradient, LN2 backward + residual, proj data
gradient, the 37-tile attention backward, qkv data gradient, LN1 backward + residual -- and the 12 weight /
bias / LayerNorm gradients are read from the flat gradient after the step (a bias gradient -- a column sum
that can cancel -- relative to the column sums of |dY| its fp32 accumulation sees).  Each op is re-computed by the
oracle (oracle/ref.py: the reference's Block at the kernels' rounding points) in float64 from the device's
OWN operands, so each comparison sees one op's rounding only.  The long-sequence attention forward takes
its softmax over 128-key chunks with a running max, so its bf16(P) rounding point is relative to that
running max: the oracle's attn_fwd_bf16_online restates exactly that.

Bars (relative L2), the F1 test's (tests/test_gpu_blocks.py): 1e-5 for fp32 outputs, 3e-4 for bf16 outputs,
1e-3 for the attention backward (two internal rounding points, bf16(P) and bf16(dS)); bf16(dY) and
bf16(dxm) bit-exact.  A 5e-3 systematic error in any kernel fails by more than an order of magnitude.

test_attention_long_vs_contract pins es_attn_fwd / es_attn_bwd at T = 577 (and a ragged T = 300) against the
same bf16-contract oracle, directly, at the op bars (the kernel tests of test_gpu_kernels.py compare them
with fp32 autograd at 2e-2 / 3e-2).
"""
import json
import os

import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
F32, B16, ATT = 1e-5, 3e-4, 1e-3


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-300)).item()


def _dump(name, rec):
    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", name), "w") as f:
        json.dump(rec, f, indent=1)


def test_s1_transformer_ops_teacher_forced():
    from endossl import conformer as cf
    from endossl.conformer import ConformerConfig, NativeConformer
    from endossl.semiformer import SemiFormer
    from endossl.utils import AttrDict
    B, MU, S, C = 1, 7, 384, 23
    model = NativeConformer(ConformerConfig(img_size=S, channel_ratio=4, embed_dim=768, depth=12, heads=12), seed=0)
    tr = SemiFormer(model, device=DEV)
    tr.get_dataloader((None, None), None)
    tr.get_config(AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=S, TARGET_NAME="target"),
                           MODEL=AttrDict(NAME="conformer", NUM_CLASSES=C),
                           TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                          EVAL_STEP_SUP=0, CLS_WEIGHT=False, THRES=0.5, T=1.0, LAMBDA_U=1.0,
                                          EPOCHS=1, WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8,
                                          SCH_NAME="const")))
    g = torch.Generator(device=DEV).manual_seed(9)
    x, y = torch.randn(B, 3, S, S, generator=g, device=DEV), torch.randint(0, C, (B,), generator=g, device=DEV)
    batch = ((x, y), ((torch.randn(B * MU, 3, S, S, generator=g, device=DEV),
                       torch.randn(B * MU, 3, S, S, generator=g, device=DEV)), None))
    m = tr.model
    cfg = m.cfg
    D, H, T = cfg.dim, cfg.heads, cfg.T
    assert (D, H, T) == (768, 12, 577)
    w0 = {k: v.detach().to(torch.float64).clone() for k, v in m.named_parameters()}
    cap = {"fwd": {}, "bwd": {}}

    def hook(kind, pre, n, *ts):
        # the token buffers are padded to 256 rows; keep the n * T live rows
        cap[kind][pre] = (n,) + tuple(t.detach()[:n * T].clone() if t.dim() == 2 else t.detach().clone() for t in ts)

    cf.BLOCK_CAPTURE = hook
    try:
        tr.step(batch)
        torch.cuda.synchronize()
    finally:
        cf.BLOCK_CAPTURE = None
    assert len(cap["fwd"]) == 12 and set(cap["bwd"]) == set(cap["fwd"]), sorted(cap["fwd"])

    rb, eps = ref._rb, cf.LN_EPS
    rec, bars = {}, {}

    def chk(key, dev, want, bar, denom=None):
        if denom is None:
            rec[key] = _rel(dev, want)
        else:  # relative to the magnitude the fp32 sum accumulates (a bias gradient cancels)
            rec[key] = ((dev.double() - want.double()).norm() / denom.double().norm().clamp_min(1e-300)).item()
        bars[key] = bar

    def ln(xx, pre, which):
        xh, rstd = ref._ln_stats(xx, eps)
        return xh, rstd, xh * w0[pre + which + ".weight"] + w0[pre + which + ".bias"]

    for pre in cap["fwd"]:
        n, xt, h1, qkv, o, lse, xmid, h2, gd, act, out = cap["fwd"][pre]
        f = lambda t: t.double()  # noqa: E731
        x, h1, qkv, o, xmid, h2, gd, act, out = map(f, (xt, h1, qkv, o, xmid, h2, gd, act, out))
        lse = lse[:n * H * T].double().view(n, H, T, 1)
        W = lambda nm: rb(w0[pre + nm + ".weight"])  # noqa: E731
        bias = lambda nm: w0[pre + nm + ".bias"]  # noqa: E731
        k = pre[:-1].replace(".trans_block", "")  # trans_1, conv_trans_2 .. conv_trans_12
        xh1, r1, y1 = ln(x, pre, "norm1")
        chk(f"{k}.op.ln1", h1, rb(y1), B16)
        chk(f"{k}.op.qkv", qkv, rb(h1 @ W("attn.qkv").T + bias("attn.qkv")), B16)
        o_ref, lse_ref = ref.attn_fwd_bf16_online(qkv, n, T, H)  # the long forward's rounding points
        chk(f"{k}.op.attn_o", o, o_ref, B16)
        chk(f"{k}.op.attn_lse", lse, lse_ref, F32)
        chk(f"{k}.op.proj_resid", xmid, x + (o @ W("attn.proj").T + bias("attn.proj")), F32)
        xh2, r2, y2 = ln(xmid, pre, "norm2")
        chk(f"{k}.op.ln2", h2, rb(y2), B16)
        z = h2 @ W("mlp.fc1").T + bias("mlp.fc1")
        chk(f"{k}.op.fc1_gelu", act, rb(ref._gelu_exact(z)), B16)
        chk(f"{k}.op.fc1_gelu_grad", gd, rb(ref._gelu_grad(z)), B16)
        chk(f"{k}.op.fc2_resid", out, xmid + (act @ W("mlp.fc2").T + bias("mlp.fc2")), F32)
        # reverse pass, each op from the device's own inputs
        _, dout, dxb, dpre, dh, dxm, dxmb, do, dqkv, dh2, dx = cap["bwd"][pre]
        dout, dxb, dpre, dh, dxm, dxmb, do, dqkv, dh2, dx = map(f, (dout, dxb, dpre, dh, dxm, dxmb, do, dqkv, dh2, dx))
        assert torch.equal(dxb, rb(dout)), pre
        assert torch.equal(dxmb, rb(dxm)), pre
        chk(f"{k}.op.fc2_dgrad_x_gelu_grad", dpre, rb((dxb @ W("mlp.fc2")) * gd), B16)
        chk(f"{k}.op.fc1_dgrad", dh, rb(dpre @ W("mlp.fc1")), B16)
        dln2, dg2, db2 = ref._ln_bwd(dh, xh2, r2, w0[pre + "norm2.weight"])
        chk(f"{k}.op.ln2_bwd_resid", dxm, dln2 + dout, F32)
        chk(f"{k}.op.proj_dgrad", do, rb(dxmb @ W("attn.proj")), B16)
        chk(f"{k}.op.attn_bwd", dqkv, ref.attn_bwd_bf16(qkv, o, lse, do, n, T, H), ATT)
        chk(f"{k}.op.qkv_dgrad", dh2, rb(dqkv @ W("attn.qkv")), B16)
        dln1, dg1, db1 = ref._ln_bwd(dh2, xh1, r1, w0[pre + "norm1.weight"])
        chk(f"{k}.op.ln1_bwd_resid", dx, dln1 + dxm, F32)
        gw = {"mlp.fc2.weight": dxb.T @ act, "mlp.fc2.bias": dxb.sum(0), "mlp.fc1.weight": dpre.T @ h2,
              "mlp.fc1.bias": dpre.sum(0), "norm2.weight": dg2, "norm2.bias": db2, "attn.proj.weight": dxmb.T @ o,
              "attn.proj.bias": dxmb.sum(0), "attn.qkv.weight": dqkv.T @ h1, "attn.qkv.bias": dqkv.sum(0),
              "norm1.weight": dg1, "norm1.bias": db1}
        absum = {"mlp.fc2.bias": dxb.abs().sum(0), "mlp.fc1.bias": dpre.abs().sum(0),
                 "attn.proj.bias": dxmb.abs().sum(0), "attn.qkv.bias": dqkv.abs().sum(0)}
        for name, v in gw.items():
            chk(f"{k}.op.grad.{name}", m.gview(pre + name).view(v.shape), v, F32, absum.get(name))
        torch.cuda.empty_cache()
    worst = {}
    for key, v in rec.items():
        c = "*." + key.split(".", 1)[1]
        worst[c] = max(worst.get(c, 0.0), v)
    rec["worst"] = worst
    rec["shape"] = {"images": B + 2 * B * MU, "tokens": T, "dim": D, "heads": H, "rows": (B + 2 * B * MU) * T}
    _dump("s1_op_parity_metrics.json", rec)
    print("worst per op:", json.dumps({k: f"{v:.2e}" for k, v in sorted(worst.items())}))
    bad = {k: (v, bars[k]) for k, v in rec.items() if k in bars and v > bars[k]}
    assert not bad, f"above the bar: {bad}"


@pytest.mark.parametrize("n,T,H", [(2, 577, 12), (3, 300, 4)])
def test_attention_long_vs_contract(n, T, H):
    """es_attn_fwd / es_attn_bwd at the long-sequence sizes (attn_fwd_long and the 37-tile / 19-tile
    backward) against the bf16-contract oracle in float64: o and dqkv at the op bars."""
    from endossl._lib import call, ptr, stream
    torch.manual_seed(T + H)
    D = H * 64
    Mp = (n * T + 255) // 256 * 256
    qkv = torch.zeros(Mp, 3 * D, dtype=torch.bfloat16, device=DEV)
    qkv[:n * T] = torch.randn(n * T, 3 * D, device=DEV).bfloat16()
    dout = torch.zeros(Mp, D, dtype=torch.bfloat16, device=DEV)
    dout[:n * T] = torch.randn(n * T, D, device=DEV).bfloat16()
    o = torch.zeros(Mp, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(n * H * T, device=DEV)
    call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 64 ** -0.5, stream())
    dqkv = torch.zeros_like(qkv)
    delta = torch.zeros(n * H * T, device=DEV)
    call("es_attn_bwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), ptr(delta), ptr(dout), D, ptr(dqkv), 3 * D, n, T, H,
         64 ** -0.5, stream())
    torch.cuda.synchronize()
    q64 = qkv[:n * T].double()
    o_ref, lse_ref = ref.attn_fwd_bf16_online(q64, n, T, H)
    assert _rel(o[:n * T], o_ref) <= B16
    assert _rel(lse.view(n, H, T, 1), lse_ref) <= F32
    d_ref = ref.attn_bwd_bf16(q64, o[:n * T].double(), lse.double().view(n, H, T, 1), dout[:n * T].double(), n, T, H)
    assert _rel(dqkv[:n * T], d_ref) <= ATT
    assert torch.all(dqkv[n * T:] == 0)
