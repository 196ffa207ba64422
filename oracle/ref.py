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


def vit_features(p, x, cfg, bf16=False):
    """The ViT trunk up to the final LayerNorm, CLS token only: the 384-d `fts` of ModelwEmb
    (code/models/custom_model.py:207-213 over a ViT backbone).  Rounding points as
    in vit_forward."""
    return _trunk(p, x, cfg, bf16)[:, 0]


def vit_forward(p, x, cfg, bf16=False):
    """timm VisionTransformer.forward with conformer.Block blocks (code/models/conformer.py:27-72).

    bf16=False: the reference arithmetic in fp32.
    bf16=True : the same arithmetic with the MI355X path's rounding points applied -- GEMM operands
    (images, LN outputs, qkv, unnormalised softmax numerators, attention output, GELU output and
    every GEMM weight) rounded to bf16; accumulation, LN/softmax statistics, the residual stream,
    biases and the CLS head stay fp32.  This is the numerical contract of the bf16 kernels; the
    difference between the two modes is the bf16 error envelope the parity tests report.
    """
    t = _trunk(p, x, cfg, bf16)
    return F.linear(t[:, 0], p["head.weight"], p["head.bias"])


def _trunk(p, x, cfg, bf16):
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
    return F.layer_norm(t, (D,), p["norm.weight"], p["norm.bias"], cfg.eps)


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


# ------------------------------------------------------------------------------------ CoMatch
DROP_P = 0.2  # build_head's Dropout(0.2) (code/models/custom_model.py:113)


def emb_param_shapes(cfg, low_dim):
    """ModelwEmb-style parameters over the ViT trunk: the trunk in timm order (no `head`), then
    fc = build_head(D, C, is_complex=True) (code/models/custom_model.py:110-116: 0 Linear(D, D/4),
    1 ReLU, 2 Dropout, 3 BatchNorm1d, 4 Linear(D/4, C)) and head_emb (:201-205: 0 Linear(D, 3L),
    1 LeakyReLU(0.1), 2 Linear(3L, L), 3 Normalize)."""
    D, C, L, Fh = cfg.dim, cfg.num_classes, low_dim, cfg.dim // 4
    trunk = [s for s in param_shapes(cfg) if not s[0].startswith("head.")]
    return trunk + [("fc.0.weight", (Fh, D)), ("fc.0.bias", (Fh,)), ("fc.3.weight", (Fh,)), ("fc.3.bias", (Fh,)),
                    ("fc.4.weight", (C, Fh)), ("fc.4.bias", (C,)), ("head_emb.0.weight", (3 * L, D)),
                    ("head_emb.0.bias", (3 * L,)), ("head_emb.2.weight", (L, 3 * L)), ("head_emb.2.bias", (L,))]


BN_BUFFERS = ("fc.3.running_mean", "fc.3.running_var", "fc.3.num_batches_tracked")


def emb_heads(p, bufs, fts, drop_keep, train=True):
    """fc and head_emb of ModelwEmb on the features (code/models/custom_model.py:110-116,136-145,
    201-213).  drop_keep: uint8/bool [N, D/4] keep-mask of the Dropout (replayed, since the reference
    draws it from torch's CPU generator); BatchNorm1d in training mode updates `bufs` in place."""
    h = F.relu(F.linear(fts, p["fc.0.weight"], p["fc.0.bias"]))
    if train:
        h = h * drop_keep.to(h.dtype) * (1.0 / (1.0 - DROP_P))
    h = F.batch_norm(h, bufs["fc.3.running_mean"], bufs["fc.3.running_var"], p["fc.3.weight"], p["fc.3.bias"],
                     training=train, momentum=0.1, eps=1e-5)
    if train:
        bufs["fc.3.num_batches_tracked"] += 1
    logits = F.linear(h, p["fc.4.weight"], p["fc.4.bias"])
    e = F.leaky_relu(F.linear(fts, p["head_emb.0.weight"], p["head_emb.0.bias"]), 0.1)
    v = F.linear(e, p["head_emb.2.weight"], p["head_emb.2.bias"])
    z = v.div(v.pow(2).sum(1, keepdim=True).pow(0.5))
    return logits, z


class CoMatchRef:
    """One-step restatement of CoMatch.train_one's body (code/comatch.py:141-231): 4-way concat,
    poly-CE, distribution alignment over <= 32 batch means, memory smoothing against the bank,
    gated bank write, contrastive loss on the pseudo-label graph, focal unsupervised loss, Adam,
    EMA over parameters and BatchNorm buffers."""

    def __init__(self, params, bufs, cfg, low_dim, num_classes, queue_size, class_weights=None, thres=0.95,
                 lambda_u=1.0, lambda_c=1.0, lr=1e-3, ema_decay=0.999, bf16=False):
        self.cfg, self.bf16, self.L, self.C = cfg, bf16, low_dim, num_classes
        self.names = [n for n, _ in emb_param_shapes(cfg, low_dim)]
        self.p = {k: params[k].detach().clone().float().requires_grad_(True) for k in self.names}
        self.bufs = {k: bufs[k].detach().clone() for k in BN_BUFFERS}
        self.ema = {k: params[k].detach().clone().float() for k in self.names}
        self.ema.update({k: bufs[k].detach().clone() for k in BN_BUFFERS})
        self.cw, self.thres, self.lambda_u, self.lambda_c, self.decay = class_weights, thres, lambda_u, lambda_c, ema_decay
        self.opt = torch.optim.Adam([self.p[k] for k in self.names], lr=lr, betas=(0.9, 0.999), eps=1e-8,
                                    weight_decay=0)
        # code/comatch.py:30-39,90-96
        self.alpha, self.temperature, self.contrast_th, self.gamma = 0.9, 0.2, 0.8, 2
        self.queue_size = queue_size
        self.queue_feats = torch.zeros(queue_size, low_dim)
        self.queue_probs = torch.zeros(queue_size, num_classes)
        self.queue_ptr = 0
        self.prob_list = []

    def step(self, x, y, uw, us0, us1, drop_keep):
        bt, btu = x.shape[0], uw.shape[0]
        imgs = torch.cat([x, uw, us0, us1], dim=0)
        fts = vit_features(self.p, imgs, self.cfg, bf16=self.bf16)
        logits, feats = emb_heads(self.p, self.bufs, fts, drop_keep, train=True)
        r = self.losses(logits, feats, y, bt, btu)
        loss = r["loss_t"]
        self.opt.zero_grad()
        loss.backward()
        grads = {k: self.p[k].grad.detach().clone() for k in self.names}
        self.opt.step()
        state = {k: self.p[k].detach() for k in self.names}
        state.update(self.bufs)
        ema_update(self.ema, state, self.decay)
        r.update({"logits": logits.detach(), "fts": fts.detach(), "z": feats.detach(), "grads": grads})
        return r

    def losses(self, logits, feats, y, bt, btu):
        """code/comatch.py:150-222 on the model outputs (logits [n, C], feats = z [n, L]): poly-CE,
        DA (appends to prob_list), memory smoothing, gated bank write, contrastive + focal losses.
        Returns the float values plus the differentiable total `loss_t`."""
        logits_x = logits[:bt]
        logits_u_w, logits_u_s0, _ = torch.split(logits[bt:], btu)
        feats_x = feats[:bt]
        feats_u_w, feats_u_s0, feats_u_s1 = torch.split(feats[bt:], btu)
        loss_x = poly_ce(logits_x, y, self.cw)
        with torch.no_grad():
            probs = torch.softmax(logits_u_w.detach(), dim=1)
            self.prob_list.append(probs.mean(0))
            if len(self.prob_list) > 32:
                self.prob_list.pop(0)
            prob_avg = torch.stack(self.prob_list, dim=0).mean(0)
            probs = probs / prob_avg
            probs = probs / probs.sum(dim=1, keepdim=True)
            probs_orig = probs.clone()
            fw = feats_u_w.detach()
            A = torch.exp(torch.mm(fw, self.queue_feats.t()) / self.temperature)
            A = A / A.sum(1, keepdim=True)
            probs = self.alpha * probs + (1 - self.alpha) * torch.mm(A, self.queue_probs)
            scores, lbs = torch.max(probs, dim=1)
            mask = scores.ge(self.thres).float()
            feats_w = torch.cat([fw, feats_x.detach()], dim=0)
            onehot = torch.zeros(bt, self.C).scatter(1, y.view(-1, 1), 1)
            probs_w = torch.cat([probs_orig, onehot], dim=0)
            n = bt + btu
            if n == self.queue_size:
                self.queue_feats[self.queue_ptr:self.queue_ptr + n, :] = feats_w
                self.queue_probs[self.queue_ptr:self.queue_ptr + n, :] = probs_w
                self.queue_ptr = (self.queue_ptr + n) % self.queue_size
        sim = torch.exp(torch.mm(feats_u_s0, feats_u_s1.t()) / self.temperature)
        sim_probs = sim / sim.sum(1, keepdim=True)
        Q = torch.mm(probs, probs.t())
        Q.fill_diagonal_(1)
        Q = Q * (Q >= self.contrast_th).float()
        Q = Q / Q.sum(1, keepdim=True)
        loss_contrast = -(torch.log(sim_probs + 1e-7) * Q).sum(1).mean()
        logp = -torch.sum(F.log_softmax(logits_u_s0, dim=1) * probs, dim=1) * mask
        pp = torch.exp(-logp)
        loss_u = ((1 - pp) ** self.gamma * logp).mean()
        loss = loss_x + self.lambda_u * loss_u + self.lambda_c * loss_contrast
        return {"lx": loss_x.item(), "lu": loss_u.item(), "lc": loss_contrast.item(), "loss": loss.item(),
                "probs": probs, "probs_orig": probs_orig, "mask": mask, "pseudo_label": lbs, "loss_t": loss}


# ------------------------------------------------------------------ one ViT block, bf16 contract
# The per-block restatement the teacher-forced parity test (tests/test_gpu_blocks.py) holds the
# production kernels to.  Arithmetic: code/models/conformer.py:8-72 (Mlp :13-23 with exact GELU,
# Attention :35-50 with scale hd^-0.5, Block :53-72 pre-norm residual, LN eps 1e-6).  Rounding points
# (the numerical contract of the bf16 kernels, forward and backward): every GEMM / attention operand
# is a bf16 value (LN outputs, qkv, the unnormalised softmax numerators bf16(e) in P.V, the attention
# output, GELU output, every weight, and in the backward the output gradients bf16(dY), bf16(dY*GELU'),
# bf16(d LN-output), bf16(d attention-output), bf16(P) / bf16(dS) inside the attention backward and the
# attention input gradient dqkv); GELU'(pre) is kept as a bf16 value; accumulation, LN / softmax
# statistics, the residual stream and its gradient, biases and their gradients stay fp32.  The
# functions keep the dtype of their inputs: float32 on the CPU is the oracle as specified; float64
# (e.g. on a device, for BASELINE-size batches) only removes accumulation-order noise.
ROUND = True  # tests switch the rounding points off to check the reverse pass against autograd


def _rb(t):
    """Round to bf16, keep the dtype (identity when ROUND is off)."""
    return t.to(torch.bfloat16).to(t.dtype) if ROUND else t


def _gelu_exact(x):
    return 0.5 * x * (1.0 + torch.erf(x * 0.7071067811865476))


def _gelu_grad(x):
    return 0.5 * (1.0 + torch.erf(x * 0.7071067811865476)) + x * torch.exp(-0.5 * x * x) * 0.3989422804014327


def _ln_stats(x, eps):
    mean = x.mean(-1, keepdim=True)
    var = ((x - mean) ** 2).mean(-1, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    return (x - mean) * rstd, rstd


def _ln_bwd(dy, xhat, rstd, w):
    """d LayerNorm: dx from dy (the bf16 values the kernel reads), xhat, rstd; dw, db as column sums."""
    g = dy * w
    dx = rstd * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).mean(-1, keepdim=True))
    return dx, (dy * xhat).sum(0), dy.sum(0)


def attn_fwd_bf16(qkv, n, T, H):
    """softmax(q k^T hd^-0.5) v per image-head (code/models/conformer.py:41-50) at the kernels'
    rounding points: qkv bf16 values [n*T, 3*H*64] (column order [3][H][64]); the unnormalised
    numerators e = exp(s - max) enter P.V as bf16(e), the sum l in full precision; o = bf16(P.V / l)
    [n*T, H*64]; lse = max + log(l) [n, H, T, 1] (what the reverse pass recomputes P from)."""
    q, k, v = qkv.view(n, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-2, -1)) * 64 ** -0.5
    mx = s.amax(-1, keepdim=True)
    e = torch.exp(s - mx)
    l = e.sum(-1, keepdim=True)
    o = _rb(((_rb(e) @ v) / l).transpose(1, 2).reshape(n * T, H * 64))
    return o, mx + torch.log(l)


def attn_fwd_bf16_online(qkv, n, T, H, chunk=128):
    """attn_fwd_bf16 at the rounding points of the long-sequence forward (T > 256, csrc/attention.hip
    fwd_long_chunk): the same softmax(q k^T hd^-0.5) v (code/models/conformer.py:41-50), taken over key
    chunks of `chunk` keys with a running max m -- per chunk P = exp(s - m_running) enters P.V as bf16(P),
    o and the unrounded sum l are rescaled by exp(m_old - m_new) when the max grows; o = bf16(o / l),
    lse = m + log(l).  Equal to attn_fwd_bf16 in exact arithmetic; the bf16(P) rounding is taken relative
    to the running max instead of the row max."""
    q, k, v = qkv.view(n, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-2, -1)) * 64 ** -0.5
    m = torch.full(s.shape[:-1] + (1,), -float("inf"), dtype=s.dtype, device=s.device)
    l = torch.zeros_like(m)
    o = torch.zeros(q.shape, dtype=s.dtype, device=s.device)
    for c0 in range(0, T, chunk):
        sc = s[..., c0:c0 + chunk]
        mn = torch.maximum(m, sc.amax(-1, keepdim=True))
        alpha = torch.exp(m - mn)
        e = torch.exp(sc - mn)
        o = o * alpha + _rb(e) @ v[..., c0:c0 + chunk, :]
        l = l * alpha + e.sum(-1, keepdim=True)
        m = mn
    return _rb((o / l).transpose(1, 2).reshape(n * T, H * 64)), m + torch.log(l)


def attn_bwd_bf16(qkv, o, lse, do, n, T, H):
    """Reverse pass of attn_fwd_bf16 (flash-style recomputation): P = exp(s - lse), delta =
    rowsum(dO * O), dS = P (dO v^T - delta); dV = bf16(bf16(P)^T dO), dK = bf16(bf16(dS)^T q * scale),
    dQ = bf16(bf16(dS) k * scale) -> dqkv [n*T, 3*H*64] in qkv's column order."""
    D = H * 64
    q, k, v = qkv.view(n, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    o4 = o.view(n, T, H, 64).transpose(1, 2)
    do4 = do.view(n, T, H, 64).transpose(1, 2)
    scale = 64 ** -0.5
    P = torch.exp((q @ k.transpose(-2, -1)) * scale - lse)
    delta = (do4 * o4).sum(-1, keepdim=True)
    dS = P * (do4 @ v.transpose(-2, -1) - delta)
    dSb = _rb(dS)
    dq = _rb((dSb @ k) * scale)
    dk = _rb((dSb.transpose(-2, -1) @ q) * scale)
    dv = _rb(_rb(P).transpose(-2, -1) @ do4)
    return torch.stack((dq, dk, dv)).permute(1, 3, 0, 2, 4).reshape(n * T, 3 * D)


def block_fwd_bf16(p, i, x, n, cfg):
    """Block i of the ViT (code/models/conformer.py:70-72: x + attn(norm1(x)), then + mlp(norm2(.)))
    over n images of cfg.T tokens, x [n*T, D] (residual stream, fp32 / fp64).  Returns (out, cache)."""
    b = f"blocks.{i}."
    D, H, T = cfg.dim, cfg.heads, cfg.T
    xh1, r1 = _ln_stats(x, cfg.eps)
    h1 = _rb(xh1 * p[b + "norm1.weight"] + p[b + "norm1.bias"])
    qkv = _rb(h1 @ _rb(p[b + "attn.qkv.weight"]).T + p[b + "attn.qkv.bias"])
    o, lse = attn_fwd_bf16(qkv, n, T, H)
    xmid = x + (o @ _rb(p[b + "attn.proj.weight"]).T + p[b + "attn.proj.bias"])
    xh2, r2 = _ln_stats(xmid, cfg.eps)
    h2 = _rb(xh2 * p[b + "norm2.weight"] + p[b + "norm2.bias"])
    pre = h2 @ _rb(p[b + "mlp.fc1.weight"]).T + p[b + "mlp.fc1.bias"]
    act = _rb(_gelu_exact(pre))
    out = xmid + (act @ _rb(p[b + "mlp.fc2.weight"]).T + p[b + "mlp.fc2.bias"])
    cache = dict(xh1=xh1, r1=r1, h1=h1, qkv=qkv, lse=lse, o=o, xh2=xh2, r2=r2, h2=h2, gd=_rb(_gelu_grad(pre)),
                 act=act)
    return out, cache


def block_bwd_bf16(p, i, cache, dy, n, cfg):
    """Reverse pass of block_fwd_bf16 given dy = d(loss)/d(out) [n*T, D] (fp32 values), at the bf16
    kernels' rounding points (see above; attention backward as flash-style recomputation from lse:
    P = exp(s - lse), delta = rowsum(dO * O)).  Returns (dx, {parameter name: gradient})."""
    b = f"blocks.{i}."
    D, H, T = cfg.dim, cfg.heads, cfg.T
    c = cache
    g = {}
    dyb = _rb(dy)
    dpre = _rb((dyb @ _rb(p[b + "mlp.fc2.weight"])) * c["gd"])
    g[b + "mlp.fc2.weight"], g[b + "mlp.fc2.bias"] = dyb.T @ c["act"], dyb.sum(0)
    dh2 = _rb(dpre @ _rb(p[b + "mlp.fc1.weight"]))
    g[b + "mlp.fc1.weight"], g[b + "mlp.fc1.bias"] = dpre.T @ c["h2"], dpre.sum(0)
    dx2, g[b + "norm2.weight"], g[b + "norm2.bias"] = _ln_bwd(dh2, c["xh2"], c["r2"], p[b + "norm2.weight"])
    dxm = dx2 + dy
    dxmb = _rb(dxm)
    do = _rb(dxmb @ _rb(p[b + "attn.proj.weight"]))
    g[b + "attn.proj.weight"], g[b + "attn.proj.bias"] = dxmb.T @ c["o"], dxmb.sum(0)
    dqkv = attn_bwd_bf16(c["qkv"], c["o"], c["lse"], do, n, T, H)
    dh1 = _rb(dqkv @ _rb(p[b + "attn.qkv.weight"]))
    g[b + "attn.qkv.weight"], g[b + "attn.qkv.bias"] = dqkv.T @ c["h1"], dqkv.sum(0)
    dx1, g[b + "norm1.weight"], g[b + "norm1.bias"] = _ln_bwd(dh1, c["xh1"], c["r1"], p[b + "norm1.weight"])
    return dx1 + dxm, g


def embed_fwd_bf16(p, x, cfg):
    """PatchEmbed Conv2d(3, D, 16, 16) on bf16 pixels and weights + cat(cls) + pos_embed (timm
    VisionTransformer.forward_features; code/models/conformer.py:420,430) -> [n*T, D]."""
    n = x.shape[0]
    t = F.conv2d(_rb(x), _rb(p["patch_embed.proj.weight"]), p["patch_embed.proj.bias"], stride=cfg.patch)
    t = torch.cat((p["cls_token"].expand(n, -1, -1), t.flatten(2).transpose(1, 2)), dim=1) + p["pos_embed"]
    return t.reshape(n * cfg.T, cfg.dim)


def head_fwd(p, x_cls, cfg):
    """Final LayerNorm + Linear head on the CLS rows (fp32; code/models/conformer.py:442-443)."""
    return F.linear(F.layer_norm(x_cls, (cfg.dim,), p["norm.weight"], p["norm.bias"], cfg.eps), p["head.weight"],
                    p["head.bias"])
