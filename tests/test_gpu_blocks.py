"""Teacher-forced per-block parity of the PRODUCTION bf16 kernels at the BASELINE F1 shapes.

One real FixMatch step (code/fixmatch.py:91-131) at configs[1]'s size -- ViT-S/16, B=64 labeled +
mu*B=448 weak/strong pairs, 224^2, tau at the median weak confidence so the consistency term and its
gradient are live -- on the default engine: gemm_nt_big / gemm_nt (incl. the two-workgroup 256x128
tile), the half-chip 384x192 weight-gradient tile with split-K, attn_fwd / attn_bwd <13>, the CLS-row
last block, LayerNorm fwd / bwd, all at M = 100,864 train tokens (88,256 weak).  The engine's capture
hook (Engine.capture) hands over each block's actual input and output, and in the reverse pass
d(loss)/d(block output) and d(loss)/d(block input).  Each of the 12 blocks is then re-computed by the
oracle's bf16-contract block (oracle/ref.py block_fwd_bf16 / block_bwd_bf16: the reference's Block,
code/models/conformer.py:53-72, at the kernels' rounding points) from THAT input and THAT output
gradient, so no error carries from one block into the next and the bar needs no depth envelope.

Bars (north_star: 1e-3), per block, relative L2:
  forward   ||out_dev - out_ref|| / ||out_ref - x_in||          (the block's own contribution)
  reverse   ||dx_dev - dx_ref|| / ||dx_ref - dy||, and every one of its 12 parameter gradients
  embedding x_0 vs patch conv + cls + pos; patch / pos / cls gradients from the device's d x_0
  heads    the train and weak logits vs the fp32 head on the device's final CLS rows
all <= 1e-3.  The oracle runs through torch in float64 on the device at this size (the CPU fp32 oracle
of one block is checked against it in the same test: same function, 16 host threads, a few seconds).
"""
import json
import os
import re

import pytest
import torch
import torch.nn.functional as F

from oracle import ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
BAR = 1e-3


def _rel(a, b, denom=None):
    d = (a.double() - b.double()).norm().item()
    n = (b.double() if denom is None else denom.double()).norm().item()
    return d / max(n, 1e-300)


def _trainer(m, B, MU, thres):
    from endossl.fixmatch import FixMatch
    from endossl.utils import AttrDict
    tr = FixMatch(m, device=DEV)
    cfg = AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=224, TARGET_NAME="target"),
                   MODEL=AttrDict(NAME="vit_small_patch16_224", NUM_CLASSES=23),
                   TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                  CLS_WEIGHT=False, THRES=thres, T=1.0, LAMBDA_U=1.0, EPOCHS=1, WARMUP_EPOCHS=0,
                                  DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const"))
    tr.get_dataloader((None, None), None)
    tr.get_config(cfg)
    return tr


def test_f1_blockwise_teacher_forced_parity():
    from endossl.vit import NativeViT, ViTConfig
    B, MU = 64, 7
    rcfg = ref.Cfg()
    params = ref.random_params(rcfg, seed=31, head_std=0.5)
    g = torch.Generator(device=DEV).manual_seed(12)
    x = torch.randn(B, 3, 224, 224, device=DEV, generator=g)
    y = torch.randint(0, 23, (B,), device=DEV, generator=g)
    uw = torch.randn(B * MU, 3, 224, 224, device=DEV, generator=g)
    us = torch.randn(B * MU, 3, 224, 224, device=DEV, generator=g)
    m = NativeViT(ViTConfig(), seed=0)
    m.load_state_dict({k: v.clone() for k, v in params.items()})
    m = m.to(DEV)
    eng = m.engine()
    assert eng.precision == "bf16" and eng._prune()
    eng.pack(m.flat, m.version)
    with torch.no_grad():
        pw = torch.softmax(eng.forward(m.flat, [uw], train=False), -1).max(-1).values
    tau = float(pw.median().item()) + 1e-4
    tr = _trainer(m, B, MU, tau)

    cap = {}

    def hook(kind, train, i, *ts):
        cap[(kind, bool(train), i)] = tuple(t.detach().clone() for t in ts)

    eng.capture = hook
    out = tr.step(((x, y), ((uw, us), None)))
    torch.cuda.synchronize()
    eng.capture = None
    n_tr, n_w, T, D, L = B + B * MU, B * MU, rcfg.T, rcfg.dim, rcfg.depth
    assert 0.0 < out["mask_mean"].item() < 1.0
    logits_tr = eng.acts(n_tr, True).logits.clone()
    logits_w = eng.acts(n_w, False).logits.clone()

    p64 = {k: v.to(DEV, torch.float64) for k, v in params.items()}
    rec = {"tau": tau, "mask_mean": out["mask_mean"].item(), "train_tokens": n_tr * T, "weak_tokens": n_w * T}
    worst = {}

    def note(key, val):
        rec[key] = val
        cat = re.sub(r"^block\d+", "block*", key)
        worst[cat] = max(worst.get(cat, 0.0), val)

    # ---- embedding (train rows: labeled + strong images; weak rows) and its reverse pass
    for train, imgs, nn_ in ((True, torch.cat([x, us]), n_tr), (False, uw, n_w)):
        x0 = cap[("fwd", train, 0)][0]
        e = ref.embed_fwd_bf16(p64, imgs.double(), rcfg)
        note(f"embed_fwd.{'train' if train else 'weak'}", _rel(x0, e))
    dx0 = cap[("bwd", True, 0)][0].double().view(n_tr, T, D)
    imgs = torch.cat([x, us]).double()
    patches = F.unfold(ref._rb(imgs), rcfg.patch, stride=rcfg.patch).transpose(1, 2).reshape(-1, 3 * rcfg.patch ** 2)
    dpatch = ref._rb(dx0[:, 1:].reshape(-1, D))
    gref = {"patch_embed.proj.weight": (dpatch.T @ patches).view(D, 3, rcfg.patch, rcfg.patch),
            "patch_embed.proj.bias": dpatch.sum(0), "pos_embed": dx0.sum(0).view(1, T, D),
            "cls_token": dx0[:, 0].sum(0).view(1, 1, D)}
    for k, v in gref.items():
        note(f"embed_grad.{k}", _rel(eng.view(m.flat_grad, k).view(v.shape), v))

    # ---- the 12 blocks: forward (train and weak rows) and reverse pass (train rows)
    def run_block(i, n, xin, dy=None, dev=DEV, dtype=torch.float64, pp=None):
        pp = p64 if pp is None else pp
        o, c = ref.block_fwd_bf16(pp, i, xin.to(dev, dtype), n, rcfg)
        if dy is None:
            return o, None, None
        dx, gr = ref.block_bwd_bf16(pp, i, c, dy.to(dev, dtype), n, rcfg)
        return o, dx, gr

    for i in range(L):
        last = i == L - 1
        for train in (True, False):
            n = n_tr if train else n_w
            xin, xout = cap[("fwd_cls" if last else "fwd", train, i)]
            dy = None
            if train:  # d loss / d block output: the next block's input gradient, or the head's
                if last:
                    dy = torch.zeros(n, T, D, device=DEV)
                    dy[:, 0] = cap[("dtop", True, i)][0]
                    dy = dy.view(n * T, D)
                else:
                    dy = cap[("bwd", True, i + 1)][0]
            o, dx, gr = run_block(i, n, xin, dy)
            xin64 = xin.double()
            if last:  # only the CLS rows leave the pruned last block
                o, xin64 = o.view(n, T, D)[:, 0], xin64.view(n, T, D)[:, 0]
            note(f"block{i}.fwd_{'train' if train else 'weak'}", _rel(xout, o, o - xin64))
            if train:
                dxd = cap[("bwd", True, i)][0]
                note(f"block{i}.dx", _rel(dxd, dx, dx - dy.double()))
                for k, v in gr.items():
                    note(f"block{i}.{k.split('.', 2)[2]}", _rel(eng.view(m.flat_grad, k).view(v.shape), v))
            del o, dx, gr
        torch.cuda.empty_cache()

    # ---- heads: logits from the device's final CLS rows (fp32 LayerNorm + Linear)
    for train, lg, nn_ in ((True, logits_tr, n_tr), (False, logits_w, n_w)):
        xcls = cap[("fwd_cls", train, L - 1)][1]
        note(f"head.{'train' if train else 'weak'}", _rel(lg, ref.head_fwd(p64, xcls.double(), rcfg)))

    # ---- the CPU fp32 oracle (as specified) agrees with its float64 device evaluation: block 5
    threads = min(16, len(os.sched_getaffinity(0)))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        xin = cap[("fwd", True, 5)][0]
        dy = cap[("bwd", True, 6)][0]
        pc = {k: v.float() for k, v in params.items()}
        oc, dxc, grc = run_block(5, n_tr, xin.cpu(), dy.cpu(), dev="cpu", dtype=torch.float32, pp=pc)
        og, dxg, grg = run_block(5, n_tr, xin, dy)
        rec["cpu_fp32_vs_device_f64.block5.fwd"] = _rel(oc, og.cpu(), og.cpu() - xin.cpu().double())
        rec["cpu_fp32_vs_device_f64.block5.dx"] = _rel(dxc, dxg.cpu(), dxg.cpu() - dy.cpu().double())
        rec["cpu_fp32_vs_device_f64.block5.grads"] = max(_rel(grc[k], grg[k].cpu()) for k in grc)
    finally:
        torch.set_num_threads(prev)

    rec["worst"] = worst
    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "block_parity_metrics.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print("worst per category:", json.dumps({k: f"{v:.2e}" for k, v in sorted(worst.items())}))
    for k in ("fwd", "dx", "grads"):
        assert rec[f"cpu_fp32_vs_device_f64.block5.{k}"] <= 1e-4, (k, rec[f"cpu_fp32_vs_device_f64.block5.{k}"])
    bad = {k: v for k, v in rec.items() if isinstance(v, float) and "." in k and not k.startswith("cpu_") and v > BAR}
    assert not bad, f"above the {BAR} bar: {bad}"
