"""Checkpoint interchange on the host (no GPU compute): the native optimizer's state_dict is
torch.optim.Adam's format over the reference's two param groups (code/optimizer.py:13-53), so a
reference checkpoint resumes natively and a native one resumes in the reference; the model
state_dict keys are timm's (code/fixmatch.py:181-236 saves / loads both)."""
import torch

from endossl.optimizer import NativeAdam, weight_decay_groups
from endossl.vit import NativeViT, ViTConfig


def _reference_adam(model, lr=1e-3):
    """code/optimizer.py:13-53 as the reference builds it over the same module."""
    skip = model.no_weight_decay()
    decay, no_decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (no_decay if len(p.shape) == 1 or name.endswith(".bias") or name in skip else decay).append(p)
    return torch.optim.Adam([{"params": decay}, {"params": no_decay, "weight_decay": 0.}], lr=lr,
                            betas=(0.9, 0.999), eps=1e-08, weight_decay=0)


def _tiny(seed=0, head="cls"):
    return NativeViT(ViTConfig(img_size=64, dim=128, depth=2, heads=2, num_classes=23, head=head), seed=seed)


def test_groups_match_set_weight_decay():
    m = _tiny()
    decay, no_decay = weight_decay_groups(m)
    assert "pos_embed" in no_decay and "cls_token" in no_decay and "blocks.0.attn.qkv.weight" in decay
    assert all(n.endswith(".bias") or m.get_parameter(n).dim() == 1 or n in m.no_weight_decay() for n in no_decay)
    assert len(decay) + len(no_decay) == len(list(m.parameters()))


def test_native_state_loads_into_torch_adam_and_back():
    torch.manual_seed(0)
    m = _tiny()
    opt = NativeAdam(m, lr=3e-4)
    opt.exp_avg.copy_(torch.randn_like(opt.exp_avg))
    opt.exp_avg_sq.copy_(torch.rand_like(opt.exp_avg_sq))
    opt.step_count = 7
    sd = opt.state_dict()

    ref = _reference_adam(m)
    ref.load_state_dict(sd)  # raises on any layout mismatch
    by_name = dict(m.named_parameters())
    for name, p in by_name.items():
        st = ref.state[p]
        o = m.offs[name]
        assert torch.equal(st["exp_avg"].flatten(), opt.exp_avg[o:o + p.numel()])
        assert torch.equal(st["exp_avg_sq"].flatten(), opt.exp_avg_sq[o:o + p.numel()])
        assert float(st["step"]) == 7
    assert ref.param_groups[0]["lr"] == 3e-4

    # and back: torch's state_dict re-loaded natively reproduces the flat moments
    opt2 = NativeAdam(_tiny(seed=1), lr=1e-3)
    opt2.load_state_dict(ref.state_dict())
    for name, p in by_name.items():
        o = m.offs[name]
        for buf in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(getattr(opt2, buf)[o:o + p.numel()], getattr(opt, buf)[o:o + p.numel()])
    assert opt2.step_count == 7 and opt2.param_groups[1]["lr"] == 3e-4


def test_reference_trained_state_resumes_natively():
    """A torch.optim.Adam that actually stepped over the module (as the reference does on CPU)."""
    torch.manual_seed(1)
    m = _tiny(head="emb")
    ref = _reference_adam(m)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    ref.step()
    ref.step()
    opt = NativeAdam(_tiny(head="emb"))
    opt.load_state_dict(ref.state_dict())
    assert opt.step_count == 2
    for name, p in m.named_parameters():
        o = m.offs[name]
        assert torch.equal(opt.exp_avg[o:o + p.numel()], ref.state[p]["exp_avg"].flatten())


def test_frozen_parameters_have_no_optimizer_state():
    m = _tiny()
    for p in m.parameters():
        p.requires_grad = False
    m.fc.requires_grad_(True)  # code/fixmatch.py:40-48 (IS_FREEZE)
    opt = NativeAdam(m)
    opt.step_count = 1
    sd = opt.state_dict()
    assert sum(len(g["params"]) for g in sd["param_groups"]) == 2 and len(sd["state"]) == 2
    ref = _reference_adam(m)
    ref.load_state_dict(sd)
    lo, hi = m.offs["head.weight"], m.numel
    frozen = opt.frozen_ranges()
    assert all(h <= lo for _, h in frozen) and hi > lo


def test_model_state_dict_round_trip():
    a, b = _tiny(seed=2), _tiny(seed=3)
    b.load_state_dict(a.state_dict())
    assert torch.equal(a.flat, b.flat)
    assert list(a.state_dict().keys())[:4] == ["cls_token", "pos_embed", "patch_embed.proj.weight",
                                               "patch_embed.proj.bias"]
