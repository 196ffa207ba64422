"""Teacher-forced per-conv parity of the production convolutions at BASELINE configs[4]'s shapes.

One SemiFormer step (code/semiformer.py:103-146) on Conformer-B (channel_ratio 4, embed 768, depth 12,
12 heads; code/models/conformer.py:308-309) at 384^2, B=1, mu=7 (15 images), bf16 convs on.  The
conformer module's capture hook (conformer.CAPTURE) hands over every convolution's actual input map,
output, output gradient and input gradient (and what the input-gradient buffer held before, where a
gradient sink accumulates into it); its weight / bias gradients are read from the flat gradient after
the step.  Each conv is then re-computed by its oracle from THOSE operands, in float64 on the device
(torch's native convolution, MIOpen off):
  conv_bf16.hip (every conv with channels % 32 == 0): the bf16-rounded-operand contract --
      y = conv(bf16(x), bf16(w)) + b, dx = conv^T(bf16(dy), bf16(w)), dw = sum bf16(dy) * im2col(bf16(x)),
      db = sum dy (csrc/conv_bf16.hip header);
  conv.hip (the 3-channel stem): plain fp32 operands.
Conformer-B runs with bf16 activation / gradient maps (conformer.NativeConformer.map_bf16): a conv whose
output (input gradient) is a bf16 map is compared with the oracle's result rounded once to bf16 (after
the gradient sink's fp32 add where one accumulates) -- the kernels' single rounding point.
One rounding point per output, so device and oracle differ by fp32 summation order only (plus the rare
bf16 rounding flip that order causes at a rounding boundary): every conv's
y, dx, dw within 1e-4 relative L2 (measured 3e-7, 3e-7, 2e-6 over the 96 convs of the step), db within 1e-4
of the per-channel sum of |dy| (a bias feeding a BatchNorm has a true gradient of exactly zero, so a relative
bar would measure cancellation noise) -- this replaces the model-level
"|device - fp32| <= 2 x envelope" bar of test_gpu_conformer.py for the bf16 convs.
"""
import json
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
BAR = 1e-4


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-300)).item()


def _rb(t, on):
    return t.to(torch.bfloat16).to(t.dtype) if on else t


def test_s1_per_conv_teacher_forced():
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
    w0 = {k: v.detach().clone() for k, v in m.named_parameters()}
    cap = {"fwd": {}, "bwd": {}}

    def hook(kind, wname, *ts):
        cap[kind][wname] = tuple(t.detach().clone() if torch.is_tensor(t) else t for t in ts)

    cf.CAPTURE = hook
    try:
        tr.step(batch)
        torch.cuda.synchronize()
    finally:
        cf.CAPTURE = None
    assert len(cap["fwd"]) > 60 and set(cap["bwd"]) == set(cap["fwd"]), set(cap["fwd"]) ^ set(cap["bwd"])
    rec, n16 = {}, 0
    with torch.backends.cudnn.flags(enabled=False):
        for wname, (xin, yout, spec) in cap["fwd"].items():
            bname, Cout, k, s, p, b16 = spec
            n16 += bool(b16)
            w = w0[wname].to(DEV, torch.float64)
            bias = w0[bname].to(DEV, torch.float64) if bname else None
            xc = xin.double().permute(0, 3, 1, 2)  # NHWC view -> NCHW
            xr = _rb(xc, b16)
            yr = F.conv2d(xr, _rb(w, b16), bias, stride=s, padding=p)
            rec[f"{wname}.y"] = _rel(yout.permute(0, 3, 1, 2), _rb(yr, yout.dtype == torch.bfloat16))
            dy, dx_before, dx_after = cap["bwd"][wname]
            dyc = dy.double().permute(0, 3, 1, 2)
            if dx_after is not None:
                dxr = torch.nn.grad.conv2d_input(xc.shape, _rb(w, b16), _rb(dyc, b16), stride=s, padding=p)
                if dx_before is not None:
                    dxr = dxr + dx_before.double().permute(0, 3, 1, 2)
                rec[f"{wname}.dx"] = _rel(dx_after.permute(0, 3, 1, 2), _rb(dxr, dx_after.dtype == torch.bfloat16))
            dwr = torch.nn.grad.conv2d_weight(xr, w.shape, _rb(dyc, b16), stride=s, padding=p)
            rec[f"{wname}.dw"] = _rel(m.gview(wname).view(w.shape), dwr)
            if bname:
                # relative to sum |dy| per channel: a conv bias in front of a BatchNorm (FCUUp's
                # conv_project) has an exactly-zero true gradient, so its sum is pure cancellation noise
                dbr = dyc.sum((0, 2, 3))
                rec[f"{wname}.db"] = ((m.gview(bname).double() - dbr).norm() / dyc.abs().sum((0, 2, 3)).norm()).item()
            del xc, xr, yr, dyc, dwr
    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    worst = {q: max(v for kk, v in rec.items() if kk.endswith("." + q)) for q in ("y", "dx", "dw", "db")
             if any(kk.endswith("." + q) for kk in rec)}
    with open(os.path.join(root, "gpurun_out", "conv_parity_metrics.json"), "w") as f:
        json.dump({"convs": len(cap["fwd"]), "bf16_convs": n16, "worst": worst, "per_conv": rec}, f, indent=1)
    print(f"{len(cap['fwd'])} convs ({n16} on conv_bf16.hip), worst:", json.dumps({k: f"{v:.2e}" for k, v in worst.items()}))
    assert n16 >= len(cap["fwd"]) - 2
    assert m.map_bf16 and sum(v[1].dtype == torch.bfloat16 for v in cap["fwd"].values()) >= len(cap["fwd"]) - 16
    bad = {k: v for k, v in rec.items() if v > BAR}
    assert not bad, f"above {BAR}: {bad}"
