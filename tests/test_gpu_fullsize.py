"""BASELINE configs[3] (C1) and configs[4] (S1) exercised at their own sizes on the production path,
through size-independent properties (the CPU oracle cannot run these sizes in a test's time).

C1: CoMatch.train_one's step (code/comatch.py:133-235) on ViT-S/16, B=64 labeled + 3 x mu*B=448
    unlabeled (weak, strong0, strong1), 224^2, L=64, a POPULATED 65,536-entry bank, EMA 0.999,
    lambda_u = lambda_c = 2.  Second step with tau at the median pseudo-label confidence of the first:
      * 0 < mask_mean < 1, losses finite and positive, gradients finite and non-zero;
      * distribution alignment + memory smoothing (code/comatch.py:167-185) re-derived in float64 from
        the device's own weak logits / embeddings, the DA history and the bank: smoothed probabilities
        within 1e-4, pseudo-labels equal and masks equal on every decidable row;
      * the smoothing used the bank (probs != 0.9 probs_orig), and the EMA is exactly
        0.999 * e_prev + 0.001 * w_new (code/ema.py:51-56).
S1: SemiFormer.train_one's SSL step (code/semiformer.py:103-146) on Conformer-B (channel_ratio 4,
    embed 768, depth 12, 12 heads; code/models/conformer.py:308-309) at 384^2 (577 tokens), B=1,
    mu=7 (15 images), bf16 convs:
      * 0 < mask_mean < 1 on the second step, finite losses, finite non-zero gradients;
      * every BatchNorm's running statistics finite, running_var > 0, moved from their initial values
        by the momentum-0.1 update, num_batches_tracked = 2 after two steps;
      * EMA of parameters 0.999 * e + 0.001 * w, and of the BatchNorm buffers likewise.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-300)).item()


def test_c1_full_size_step_properties():
    from endossl.comatch import CoMatch
    from endossl.comatch_model import NativeViTEmb
    from endossl.utils import AttrDict
    from endossl.vit import ViTConfig
    B, MU, L, Q, C = 64, 7, 64, 65536, 23
    model = NativeViTEmb(ViTConfig(head="emb", low_dim=L), seed=0)
    tr = CoMatch(model, device=DEV)
    cfg = AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=224, TARGET_NAME="target"),
                   MODEL=AttrDict(NAME="vit_small_patch16_224", NUM_CLASSES=C, LOW_DIM=L, TYPE_SEMI="CoMatch"),
                   TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                  CLS_WEIGHT=False, THRES=0.95, T=1.0, LAMBDA_U=2.0, LAMBDA_C=2.0, EPOCHS=1,
                                  WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const"))
    tr.get_dataloader((None, None), None)
    tr.get_config(cfg)
    tr.set_queue_size(Q)
    g = torch.Generator(device=DEV).manual_seed(5)
    # a populated bank (as after earlier epochs): unit features, peaked class rows
    tr.queue_feats.copy_(torch.nn.functional.normalize(torch.randn(Q, L, generator=g, device=DEV), dim=1))
    tr.queue_probs.copy_(torch.softmax(torch.randn(Q, C, generator=g, device=DEV) * 3, 1))
    x, y = torch.randn(B, 3, 224, 224, generator=g, device=DEV), torch.randint(0, C, (B,), generator=g, device=DEV)
    unl = tuple(torch.randn(B * MU, 3, 224, 224, generator=g, device=DEV) for _ in range(3))
    batch = ((x, y), (unl, None))
    o1 = tr.step(batch)
    torch.cuda.synchronize()
    tau = float(o1["probs"].max(1).values.median().item()) + 1e-4
    tr.config.TRAIN.THRES = tau
    hist = [h.double().clone() for h in tr.prob_list]  # the DA history the second step extends
    m = tr.model
    w1, e1 = m.flat.clone(), tr.ema_model.ema.flat.clone()
    o2 = tr.step(batch)
    torch.cuda.synchronize()
    for k in ("loss", "lx", "lu", "lc"):
        assert torch.isfinite(o2[k]).item(), k
    assert o2["lu"].item() > 0 and o2["lc"].item() > 0
    assert 0.0 < o2["mask_mean"].item() < 1.0, o2["mask_mean"].item()
    assert torch.isfinite(m.flat_grad).all().item() and float(m.flat_grad.abs().sum()) > 0
    torch.testing.assert_close(tr.ema_model.ema.flat, 0.999 * e1 + 0.001 * m.flat, rtol=1e-6, atol=1e-7)
    assert float((m.flat - w1).abs().max()) > 0

    # DA + memory smoothing re-derived from the device's own weak logits / embeddings (code/comatch.py:167-185)
    lw = o2["logits"][B:B + B * MU].double()
    zw = o2["z"][B:B + B * MU].double()
    with torch.no_grad():
        probs = torch.softmax(lw, 1)
        hist.append(probs.mean(0))
        probs = probs / torch.stack(hist[-32:]).mean(0)
        probs = probs / probs.sum(1, keepdim=True)
        probs_orig = probs.clone()
        A = torch.exp(zw @ tr.queue_feats.double().t() / 0.2)
        A = A / A.sum(1, keepdim=True)
        probs = 0.9 * probs + 0.1 * (A @ tr.queue_probs.double())
        scores, lbs = probs.max(1)
    assert _rel(o2["probs_orig"], probs_orig) <= 1e-4, _rel(o2["probs_orig"], probs_orig)
    assert _rel(o2["probs"], probs) <= 1e-4, _rel(o2["probs"], probs)
    assert (o2["probs"].double() - 0.9 * o2["probs_orig"].double()).abs().max().item() > 1e-3  # the bank was used
    top2 = probs.topk(2, 1).values
    ok = (top2[:, 0] - top2[:, 1]) > 1e-5
    okm = (scores - tau).abs() > 1e-5
    assert ok.float().mean() > 0.95 and okm.float().mean() > 0.95
    assert torch.equal(o2["pseudo_label"].long()[ok], lbs[ok])
    assert torch.equal(o2["mask"].bool()[okm], scores.ge(tau)[okm])


def test_s1_full_size_step_properties():
    from endossl.conformer import ConformerConfig, NativeConformer
    from endossl.semiformer import SemiFormer
    from endossl.utils import AttrDict
    B, MU, S, C = 1, 7, 384, 23
    ccfg = ConformerConfig(img_size=S, channel_ratio=4, embed_dim=768, depth=12, heads=12)
    assert ccfg.T == 577
    model = NativeConformer(ccfg, seed=0)
    assert model.conv_bf16
    buf0 = {k: v.detach().clone() for k, v in model.named_buffers()}
    tr = SemiFormer(model, device=DEV)
    cfg = AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=S, TARGET_NAME="target"),
                   MODEL=AttrDict(NAME="conformer", NUM_CLASSES=C),
                   TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-5, EVAL_STEP=1,
                                  EVAL_STEP_SUP=0, CLS_WEIGHT=False, THRES=0.95, T=1.0, LAMBDA_U=1.0, EPOCHS=1,
                                  WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const"))
    tr.get_dataloader((None, None), None)
    tr.get_config(cfg)
    g = torch.Generator(device=DEV).manual_seed(7)
    x, y = torch.randn(B, 3, S, S, generator=g, device=DEV), torch.randint(0, C, (B,), generator=g, device=DEV)
    batch = ((x, y), ((torch.randn(B * MU, 3, S, S, generator=g, device=DEV),
                       torch.randn(B * MU, 3, S, S, generator=g, device=DEV)), None))
    o1 = tr.step(batch)
    torch.cuda.synchronize()
    # tau at the median conv-head weak confidence: the consistency terms and their gradients are live (lr 1e-5:
    # Adam's first step moves every weight by ~lr, which at 1e-3 shifts this BatchNorm net's confidences wholesale)
    weak = o1["out_conv"][B:B + B * MU]
    tr.config.TRAIN.THRES = float(torch.softmax(weak, -1).max(-1).values.median().item()) + 1e-4
    m = tr.model
    w1, e1 = m.flat.clone(), tr.ema_model.ema.flat.clone()
    eb1 = {k: v.detach().clone() for k, v in tr.ema_model.ema.named_buffers()}
    o2 = tr.step(batch)
    torch.cuda.synchronize()
    for k in ("loss", "lx", "lu"):
        assert torch.isfinite(o2[k]).item(), k
    assert 0.0 < o2["mask_mean"].item() < 1.0, o2["mask_mean"].item()
    assert torch.isfinite(m.flat_grad).all().item() and float(m.flat_grad.abs().sum()) > 0
    torch.testing.assert_close(tr.ema_model.ema.flat, 0.999 * e1 + 0.001 * m.flat, rtol=1e-6, atol=1e-7)
    assert float((m.flat - w1).abs().max()) > 0
    nbn = 0
    for k, v in m.named_buffers():
        if k.endswith("num_batches_tracked"):
            assert int(v.item()) == int(buf0[k].item()) + 2, k
            ev = dict(tr.ema_model.ema.named_buffers())[k]
            assert int(ev.item()) == int(0.999 * eb1[k].double().item() + 0.001 * int(v.item())), k
            continue
        nbn += 1
        assert torch.isfinite(v).all().item(), k
        assert not torch.equal(v.cpu(), buf0[k]), k  # moved by the momentum-0.1 batch-statistics update
        if k.endswith("running_var"):
            assert (v > 0).all().item(), k
        ev = dict(tr.ema_model.ema.named_buffers())[k]
        torch.testing.assert_close(ev, 0.999 * eb1[k] + 0.001 * v, rtol=1e-6, atol=1e-7)
    assert nbn > 100  # every BatchNorm of the CNN branch and the FCU bridges
