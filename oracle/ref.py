"""ORACLE (test infrastructure only): CPU fp32 restatement of the reference SSL step.

Each function cites the reference code it restates.  Pinned by tests/test_oracle_golden.py
against fixtures generated from the reference (tests/golden/make_golden.py).
"""
import math

import torch
import torch.nn.functional as F


class Cfg:
    def __init__(self, img_size=224, patch=16, dim=384, depth=12, heads=6, mlp_ratio=4.0, num_classes=23, eps=1e-6):
        self.img_size, self.patch, self.dim, self.depth, self.heads = img_size, patch, dim, depth, heads
        self.hidden, self.num_classes, self.eps = int(dim * mlp_ratio), num_classes, eps
        self.np = (img_size // patch) ** 2
        self.T = self.np + 1


def param_shapes(cfg):
    """timm 0.5.4 VisionTransformer state_dict order (cls_token, pos_embed, patch_embed, blocks, norm, head)."""
    D, Hd, C = cfg.dim, cfg.hidden, cfg.num_classes
    out = [("cls_token", (1, 1, D)), ("pos_embed", (1, cfg.T, D)),
           ("patch_embed.proj.weight", (D, 3, cfg.patch, cfg.patch)), ("patch_embed.proj.bias", (D,))]
    for i in range(cfg.depth):
        b = f"blocks.{i}."
        out += [(b + "norm1.weight", (D,)), (b + "norm1.bias", (D,)), (b + "attn.qkv.weight", (3 * D, D)),
                (b + "attn.qkv.bias", (3 * D,)), (b + "attn.proj.weight", (D, D)), (b + "attn.proj.bias", (D,)),
                (b + "norm2.weight", (D,)), (b + "norm2.bias", (D,)), (b + "mlp.fc1.weight", (Hd, D)),
                (b + "mlp.fc1.bias", (Hd,)), (b + "mlp.fc2.weight", (D, Hd)), (b + "mlp.fc2.bias", (D,))]
    out += [("norm.weight", (D,)), ("norm.bias", (D,)), ("head.weight", (C, D)), ("head.bias", (C,))]
    return out


def _bf(t):
    """Round to bf16 and back (the MI355X path's GEMM-operand rounding points)."""
    return t.bfloat16().float()


def vit_forward(p, x, cfg, bf16=False):
    """timm VisionTransformer.forward with conformer.Block blocks (code/models/conformer.py:27-72).

    bf16=False: the reference arithmetic in fp32.
    bf16=True : the same arithmetic with the MI355X path's rounding points applied -- GEMM operands
    (images, LN outputs, qkv, unnormalised softmax numerators, attention output, GELU output and
    every GEMM weight) rounded to bf16; accumulation, LN/softmax statistics, the residual stream,
    biases and the CLS head stay fp32.  This is the numerical contract of the bf16 kernels; the
    difference between the two modes is the bf16 error envelope the parity tests report.
    """
    B, D, H = x.shape[0], cfg.dim, cfg.heads
    hd = D // H
    r = _bf if bf16 else (lambda t: t)
    t = F.conv2d(r(x), r(p["patch_embed.proj.weight"]), p["patch_embed.proj.bias"], stride=cfg.patch)
    t = t.flatten(2).transpose(1, 2)
    t = torch.cat((p["cls_token"].expand(B, -1, -1), t), dim=1) + p["pos_embed"]
    N = t.shape[1]
    for i in range(cfg.depth):
        b = f"blocks.{i}."
        h = r(F.layer_norm(t, (D,), p[b + "norm1.weight"], p[b + "norm1.bias"], cfg.eps))
        qkv = r(F.linear(h, r(p[b + "attn.qkv.weight"]), p[b + "attn.qkv.bias"]))
        qkv = qkv.reshape(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        attn = (q @ k.transpose(-2, -1)) * hd ** -0.5
        if bf16:
            e = torch.exp(attn - attn.amax(-1, keepdim=True))
            o = (_bf(e) @ v) / e.sum(-1, keepdim=True)
        else:
            o = attn.softmax(dim=-1) @ v
        o = r(o.transpose(1, 2).reshape(B, N, D))
        t = t + F.linear(o, r(p[b + "attn.proj.weight"]), p[b + "attn.proj.bias"])
        h = r(F.layer_norm(t, (D,), p[b + "norm2.weight"], p[b + "norm2.bias"], cfg.eps))
        h = r(F.gelu(F.linear(h, r(p[b + "mlp.fc1.weight"]), p[b + "mlp.fc1.bias"])))
        t = t + F.linear(h, r(p[b + "mlp.fc2.weight"]), p[b + "mlp.fc2.bias"])
    t = F.layer_norm(t, (D,), p["norm.weight"], p["norm.bias"], cfg.eps)
    return F.linear(t[:, 0], p["head.weight"], p["head.bias"])


def poly_ce(logits, targets, weights=None, epsilon=2.0):
    """PolyLoss(softmax=True, ce_weight, reduction='mean', epsilon) (code/loss.py:308-364)."""
    ce = F.cross_entropy(logits, targets, weight=weights, reduction="none")
    pt = torch.softmax(logits, 1).gather(1, targets.view(-1, 1)).squeeze(1)
    return torch.mean(ce + epsilon * (1 - pt))


def consistency(logits_w, logits_s, p_cutoff):
    """consistency_loss(name='ce', use_hard_labels=True) (code/loss.py:126-164).
    Returns (loss, mask_mean, pseudo_label, mask)."""
    pseudo = torch.softmax(logits_w.detach(), dim=-1)
    max_probs, max_idx = torch.max(pseudo, dim=-1)
    mask = max_probs.ge(p_cutoff).float()
    masked = F.cross_entropy(logits_s, max_idx, reduction="none") * mask
    return masked.mean(), mask.mean(), max_idx, mask


def ema_update(ema_sd, model_sd, decay):
    """ModelEMA._update (code/ema.py:51-59): copy_(decay*e + (1-decay)*m) for every entry."""
    with torch.no_grad():
        for k in ema_sd:
            e, m = ema_sd[k], model_sd[k]
            e.copy_(decay * e + (1.0 - decay) * m)


class FixMatchRef:
    """One-step restatement of FixMatch.train_one's body (code/fixmatch.py:91-131)."""

    def __init__(self, params, cfg, class_weights=None, thres=0.95, lambda_u=1.0, lr=1e-3, ema_decay=0.999,
                 bf16=False):
        self.cfg, self.bf16 = cfg, bf16
        self.names = [n for n, _ in param_shapes(cfg)]
        self.p = {k: params[k].detach().clone().float().requires_grad_(True) for k in self.names}
        self.ema = {k: params[k].detach().clone().float() for k in self.names}
        self.cw = class_weights
        self.thres, self.lambda_u, self.decay = thres, lambda_u, ema_decay
        self.opt = torch.optim.Adam([self.p[k] for k in self.names], lr=lr, betas=(0.9, 0.999), eps=1e-8,
                                    weight_decay=0)

    def step(self, x, y, uw, us):
        B = x.shape[0]
        out = vit_forward(self.p, torch.cat((x, uw, us)), self.cfg, bf16=self.bf16)
        ox = out[:B]
        ow, os_ = out[B:].chunk(2)
        lx = poly_ce(ox, y, self.cw)
        lu, mask_mean, pl, mask = consistency(ow, os_, self.thres)
        loss = lx + self.lambda_u * lu
        self.opt.zero_grad()
        loss.backward()
        grads = {k: self.p[k].grad.detach().clone() for k in self.names}
        self.opt.step()
        ema_update(self.ema, {k: self.p[k].detach() for k in self.names}, self.decay)
        return {"lx": lx.item(), "lu": lu.item(), "mask_mean": mask_mean.item(), "loss": loss.item(),
                "pseudo_label": pl, "mask": mask, "logits": out.detach(), "grads": grads}


def random_params(cfg, seed=0, std=0.02, head_std=0.02):
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in param_shapes(cfg):
        if name.endswith("norm1.weight") or name.endswith("norm2.weight") or name == "norm.weight":
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name.startswith("head.weight"):
            t = head_std * torch.randn(shape, generator=g)
        elif len(shape) >= 2 or name in ("cls_token", "pos_embed"):
            t = std * torch.randn(shape, generator=g)
        elif name == "patch_embed.proj.bias":
            t = (1.0 / math.sqrt(3 * cfg.patch * cfg.patch)) * (2 * torch.rand(shape, generator=g) - 1)
        else:
            t = 0.02 * torch.randn(shape, generator=g)
        out[name] = t.float()
    return out
