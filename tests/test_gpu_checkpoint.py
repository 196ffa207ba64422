"""Head-only training (IS_FREEZE) and checkpoint interchange on the MI355X.

  * IS_FREEZE (code/fixmatch.py:40-48, code/comatch.py:64-73, code/semiformer.py:50-56): every
    parameter outside the trainable heads is bit-for-bit unchanged by a step; the heads move; in the
    fp32 parity mode the head gradient equals the fp32 oracle's (the head gradient does not depend on
    whether the trunk is frozen).
  * save_checkpoint / load_checkpoint (code/fixmatch.py:181-236): a trainer restored from a native
    checkpoint continues bit-identically to the one that saved it; the checkpoint's optimizer entry
    is torch.optim.Adam's format (it loads into a torch Adam over the same module); evaluate_one runs
    the EMA model, whose logits match the fp32 oracle on the EMA weights (parity mode).
"""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import ref  # noqa: E402

DEV = "cuda"


class _DS:
    def __init__(self, df=None):
        self.df = df


class _DL:
    def __init__(self, items):
        self.items, self.dataset = items, _DS()

    def __iter__(self):
        return iter(self.items)

    def __len__(self):
        return len(self.items)


def _cfg(freeze, B, MU, thres=0.3, L=None, name="vit_tiny_test", semi="FixMatch"):
    from endossl.utils import AttrDict
    model = AttrDict(NAME=name, NUM_CLASSES=23, TYPE_SEMI=semi)
    if L:
        model.LOW_DIM = L
    return AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=64, TARGET_NAME="target"), MODEL=model,
                    TRAIN=AttrDict(IS_FREEZE=freeze, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                   EVAL_STEP_SUP=0, CLS_WEIGHT=False, THRES=thres, T=1.0, LAMBDA_U=1.0, LAMBDA_C=1.0,
                                   EPOCHS=2, WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8,
                                   SCH_NAME="const", FREQ_EVAL=1, SAVE_CP="."))


def _batch(B, MU, n_u=2, seed=0, img=64):
    g = torch.Generator().manual_seed(seed)
    x, y = torch.randn(B, 3, img, img, generator=g), torch.randint(0, 23, (B,), generator=g)
    return (x, y), (tuple(torch.randn(B * MU, 3, img, img, generator=g) for _ in range(n_u)), None)


def _tiny_vit(seed=3, head="cls", precision="bf16"):
    from endossl.vit import NativeViT, ViTConfig
    from endossl.comatch_model import NativeViTEmb
    if head == "cls":
        m = NativeViT(ViTConfig(img_size=64, dim=128, depth=2, heads=2, num_classes=23), seed=seed)
        with torch.no_grad():
            m.head.weight.normal_(0, 0.5, generator=torch.Generator().manual_seed(seed))
    else:
        m = NativeViTEmb(ViTConfig(img_size=64, dim=128, depth=2, heads=2, num_classes=23, head="emb", low_dim=16),
                         seed=seed)
    return m.to(DEV).set_precision(precision)


def _head_ranges(m, names):
    return [(m.offs[n], m.offs[n] + m.get_parameter(n).numel()) for n in names]


def _frozen_unchanged(m, before, trainable):
    """Every parameter outside `trainable` (names) bit-identical to `before`; the trainable ones moved."""
    for name, p in m.named_parameters():
        o = m.offs[name]
        now, was = m.flat[o:o + p.numel()], before[o:o + p.numel()]
        if name in trainable:
            assert not torch.equal(now, was), f"{name} did not move"
        else:
            assert torch.equal(now, was), f"frozen {name} changed"


def test_fixmatch_is_freeze_head_only():
    from endossl.fixmatch import FixMatch
    m = _tiny_vit(precision="fp32")
    params = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    tr = FixMatch(m, device=DEV)
    tr.get_dataloader((None, None), None)
    tr.get_config(_cfg(True, 4, 2))
    assert [n for n, p in m.named_parameters() if p.requires_grad] == ["head.weight", "head.bias"]
    assert sum(len(g) for g in tr.optimizer._group_names) == 2
    before = m.flat.clone()
    (x, y), ((uw, us), _) = _batch(4, 2)
    out = tr.step(((x, y), ((uw, us), None)))
    torch.cuda.synchronize()
    _frozen_unchanged(m, before, {"head.weight", "head.bias"})
    # the head gradient is the unfrozen step's head gradient: fp32 oracle, parity mode
    rcfg = ref.Cfg(img_size=64, patch=16, dim=128, depth=2, heads=2, num_classes=23)
    r = ref.FixMatchRef(params, rcfg, class_weights=None, thres=0.3).step(x, y, uw, us)
    for name in ("head.weight", "head.bias"):
        got = m.engine().view(m.flat_grad, name).cpu().view(r["grads"][name].shape)
        torch.testing.assert_close(got, r["grads"][name], rtol=1e-4, atol=1e-5)
    assert abs(out["lx"].item() - r["lx"]) <= 1e-5 * max(1.0, abs(r["lx"]))


def test_comatch_is_freeze_heads_only():
    from endossl.comatch import CoMatch
    m = _tiny_vit(head="emb")
    tr = CoMatch(m, device=DEV)
    tr.get_dataloader((None, None), None)
    tr.get_config(_cfg(True, 4, 2, L=16, semi="CoMatch"))
    trainable = {n for n, p in m.named_parameters() if p.requires_grad}
    assert trainable == {n for n, _ in m.named_parameters() if n.startswith(("fc.", "head_emb."))}
    before = m.flat.clone()
    lab, unl = _batch(4, 2, n_u=3)
    tr.step((lab, unl))
    torch.cuda.synchronize()
    _frozen_unchanged(m, before, trainable)
    assert m.bn_buffers()[2].item() == 1  # BatchNorm1d still in training mode (running stats updated)


def test_semiformer_is_freeze_heads_only():
    from endossl.conformer import ConformerConfig, NativeConformer
    from endossl.semiformer import SemiFormer
    m = NativeConformer(ConformerConfig(img_size=64, patch=16, base_channel=16, embed_dim=128, depth=3, heads=2,
                                        num_classes=23), seed=1)
    m = m.to(DEV)
    tr = SemiFormer(m, device=DEV)
    tr.get_dataloader((None, None), None)
    tr.get_config(_cfg(True, 2, 2, semi="SemiFormer", name="conformer"))
    trainable = {n for n, p in m.named_parameters() if p.requires_grad}
    assert trainable == {"conv_cls_head.weight", "conv_cls_head.bias", "trans_cls_head.weight", "trans_cls_head.bias"}
    before = m.flat.clone()
    lab, unl = _batch(2, 2)
    tr.step((lab, unl))
    torch.cuda.synchronize()
    _frozen_unchanged(m, before, trainable)


def test_checkpoint_round_trip_and_evaluate(tmp_path):
    from endossl.fixmatch import FixMatch
    batches = [_batch(4, 2, seed=s) for s in range(3)]
    valid = [(torch.randn(6, 3, 64, 64, generator=torch.Generator().manual_seed(50)), torch.arange(6) % 23)]

    def make():
        m = _tiny_vit(precision="fp32")
        tr = FixMatch(m, device=DEV)
        tr.get_dataloader((None, None), _DL(valid))
        tr.get_config(_cfg(False, 4, 2))
        return m, tr

    m1, t1 = make()
    t1.step(batches[0])
    t1.step(batches[1])
    t1.epoch = 1
    path = t1.save_checkpoint(str(tmp_path))
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ck) == {"ema_state_dict", "epoch", "best_valid_perf", "model_state_dict", "optimizer", "scheduler"}
    # the optimizer entry is torch.optim.Adam's own format over the module's two param groups
    from endossl.optimizer import weight_decay_groups
    cpu = _tiny_vit(precision="fp32").cpu()
    decay, no_decay = weight_decay_groups(cpu)
    tadam = torch.optim.Adam([{"params": [cpu.get_parameter(n) for n in decay]},
                              {"params": [cpu.get_parameter(n) for n in no_decay], "weight_decay": 0.}], lr=1e-3)
    tadam.load_state_dict(ck["optimizer"])

    m2, t2 = make()
    t2.load_checkpoint(path, is_train=True)
    assert torch.equal(m2.flat, m1.flat) and torch.equal(t2.ema_model.ema.flat, t1.ema_model.ema.flat)
    assert torch.equal(t2.optimizer.exp_avg_sq, t1.optimizer.exp_avg_sq) and t2.optimizer.step_count == 2
    o1, o2 = t1.step(batches[2]), t2.step(batches[2])
    torch.cuda.synchronize()
    assert o1["loss"].item() == o2["loss"].item()
    assert (m1.flat - m2.flat).abs().max().item() <= 1e-7  # only the head's fp32 atomics may reorder

    # evaluate_one: the EMA model in eval mode; its logits vs the fp32 oracle on the EMA weights
    loss, metric = t2.evaluate_one()
    ema = t2.ema_model.ema
    with torch.no_grad():
        logits = ema(valid[0][0].to(DEV)).cpu()
    rcfg = ref.Cfg(img_size=64, patch=16, dim=128, depth=2, heads=2, num_classes=23)
    want = ref.vit_forward({k: v.cpu() for k, v in ema.state_dict().items()}, valid[0][0], rcfg)
    torch.testing.assert_close(logits, want, rtol=1e-4, atol=1e-4)
    ce = torch.nn.functional.cross_entropy(want, valid[0][1]).item()
    assert math.isclose(loss.avg, ce, rel_tol=1e-4, abs_tol=1e-5)
    assert isinstance(metric, dict)
