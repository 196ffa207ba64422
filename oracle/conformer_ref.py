"""ORACLE (test infrastructure only): CPU fp32 restatement of the reference Conformer and one
SemiFormer step.

  * Conformer.forward            code/models/conformer.py:418-445 (stem, conv_1, trans_patch_conv,
                                 trans_1, ConvTransBlocks, pooled conv head, trans_norm + head)
  * ConvBlock.forward            code/models/conformer.py:107-144 (conv2(x + x_t) when fused)
  * FCUDown / FCUUp              code/models/conformer.py:152-200
  * ConvTransBlock.forward       code/models/conformer.py:338-356 (x_st + x_t: the cls row doubles)
  * Conformer.__init__ stages    code/models/conformer.py:373-416 (channels, strides, dw_stride,
                                 res_conv on the first block of a stage, last_fusion)
  * Block / Attention / Mlp      code/models/conformer.py:8-72 (the ViT-block restatement of ref.py)
  * SemiFormer.train_one SSL     code/semiformer.py:103-146 (two CE heads, two consistency losses
                                 against the conv head's weak logits, Adam, EMA over every entry)

Pinned by tests/test_oracle_golden.py against tests/golden/semiformer_step.npz, which
tests/golden/make_golden.py produces by running the reference's own SemiFormer.train_one on a
tiny Conformer.  bf16=True applies the MI355X path's rounding points: the transformer blocks'
GEMM operands, and the operands of every conv the device runs on csrc/conv_bf16.hip (both channel
counts multiples of 32); BatchNorm, the FCU LayerNorm / pooling, the heads and the 3-channel stem
conv stay fp32 as on the device.  bf16_maps=True adds the device's bf16 activation / gradient maps
(conformer.NativeConformer.map_bf16, Conformer-B): every CNN map after the stem's max-pool is rounded
to bf16 where the device stores it -- conv outputs, BatchNorm (+ residual) (+ ReLU) outputs, the
FCUDown pooled map, the FCUUp output and the upsample-add -- and so is the gradient arriving at each of
them (_RoundMap); BatchNorms fed by a bf16 conv take their batch statistics from the conv's fp32
output (the conv epilogue's statistics, es_conv2d_fwd_bf16_ex) and normalise the rounded map.
"""
import torch
import torch.nn.functional as F

from .ref import _bf, _gelu_grad, consistency, ema_update

BN_EPS_BLOCK = 1e-6   # ConvBlock / FCUUp norm_layer = partial(nn.BatchNorm2d, eps=1e-6)
BN_EPS_STEM = 1e-5    # Conformer.bn1 = nn.BatchNorm2d(64)
LN_EPS_BLOCK = 1e-6   # Block / FCUDown LayerNorm(eps=1e-6)
LN_EPS_TRANS_NORM = 1e-5  # Conformer.trans_norm = nn.LayerNorm(embed_dim)


class ConformerCfg:
    def __init__(self, img_size=224, patch=16, base_channel=64, channel_ratio=1, embed_dim=384, depth=12, heads=6,
                 mlp_ratio=4.0, num_classes=23):
        assert depth % 3 == 0
        self.img_size, self.patch, self.base, self.ratio = img_size, patch, base_channel, channel_ratio
        self.dim, self.depth, self.heads, self.num_classes = embed_dim, depth, heads, num_classes
        self.hidden = int(embed_dim * mlp_ratio)
        self.stem = img_size // 4
        self.grid = self.stem // (patch // 4)
        self.np = self.grid * self.grid
        self.T = self.np + 1


def stages(cfg):
    """(name, inplanes, outplanes, res_conv, stride, dw_stride, last_fusion) per ConvTransBlock
    (code/models/conformer.py:385-416)."""
    s1, dw = cfg.base * cfg.ratio, cfg.patch // 4
    out = []
    fin = cfg.depth // 3 + 1
    for i in range(2, fin):
        out.append((f"conv_trans_{i}", s1, s1, False, 1, dw, False))
    s2 = s1 * 2
    init, fin = fin, fin + cfg.depth // 3
    for i in range(init, fin):
        out.append((f"conv_trans_{i}", s1 if i == init else s2, s2, i == init, 2 if i == init else 1, dw // 2, False))
    s3 = s2 * 2
    init, fin = fin, fin + cfg.depth // 3
    for i in range(init, fin):
        out.append((f"conv_trans_{i}", s2 if i == init else s3, s3, i == init, 2 if i == init else 1, dw // 4,
                    i == cfg.depth))
    return out


def _bn(x, p, bufs, pre, eps, train):
    y = F.batch_norm(x, bufs[pre + "running_mean"], bufs[pre + "running_var"], p[pre + "weight"], p[pre + "bias"],
                     training=train, momentum=0.1, eps=eps)
    if train:
        bufs[pre + "num_batches_tracked"] += 1
    return y


class _RoundMap(torch.autograd.Function):
    """A bf16 map: the value rounded where the device stores it, and the gradient arriving at it."""

    @staticmethod
    def forward(ctx, x):
        return _bf(x)

    @staticmethod
    def backward(ctx, g):
        return _bf(g)


class _GeluB16(torch.autograd.Function):
    """GELU of the fp32 fc1 output under the bf16 contract: the device's fc1 epilogue writes GELU'(pre) rounded
    to bf16 beside the activation (endossl/conformer.py, EPI_GELU_D) and the backward multiplies by that stored
    value (EPI_MULAUX), so the reverse pass here uses the same rounded derivative."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return F.gelu(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * _bf(_gelu_grad(x))


def _bn_map(y32, p, bufs, pre, eps, train):
    """BatchNorm2d of a bf16 conv output stored as a bf16 map: batch statistics of the fp32 output, the
    normalisation applied to the rounded map (train); eval: running statistics on the rounded map."""
    y16 = _RoundMap.apply(y32)
    if not train:
        return _bn(y16, p, bufs, pre, eps, False)
    n = y32.numel() // y32.shape[1]
    mean = y32.mean((0, 2, 3))
    var = y32.var((0, 2, 3), unbiased=False)
    with torch.no_grad():
        rm, rv = bufs[pre + "running_mean"], bufs[pre + "running_var"]
        rm.mul_(0.9).add_(0.1 * mean.detach())
        rv.mul_(0.9).add_(0.1 * var.detach() * n / max(n - 1, 1))
        bufs[pre + "num_batches_tracked"] += 1
    sh = (1, -1, 1, 1)
    return (y16 - mean.view(sh)) * torch.rsqrt(var.view(sh) + eps) * p[pre + "weight"].view(sh) + \
        p[pre + "bias"].view(sh)


def _ident(x):
    return x


def conv2d(x, w, b=None, stride=1, padding=0, bf16=False):
    """F.conv2d; bf16=True rounds both operands to bf16 where the device takes the bf16 kernels
    (es_conv2d_bf16_eligible: Cin and Cout multiples of 32), accumulation fp32 as on the device."""
    if bf16 and w.shape[0] % 32 == 0 and w.shape[1] % 32 == 0:
        x, w = _bf(x), _bf(w)
    return F.conv2d(x, w, b, stride=stride, padding=padding)


def conv_block(p, bufs, pre, x, stride, res_conv, x_t=None, train=True, bf16=False, maps=False):
    """ConvBlock.forward (code/models/conformer.py:107-144); returns (x, x2).  maps: bf16 maps."""
    rm, bn = (_RoundMap.apply, _bn_map) if maps else (_ident, _bn)
    residual = x
    x = rm(F.relu(bn(conv2d(x, p[pre + "conv1.weight"], bf16=bf16), p, bufs, pre + "bn1.", BN_EPS_BLOCK, train)))
    x = conv2d(x if x_t is None else rm(x + x_t), p[pre + "conv2.weight"], stride=stride, padding=1, bf16=bf16)
    x2 = rm(F.relu(bn(x, p, bufs, pre + "bn2.", BN_EPS_BLOCK, train)))
    x = bn(conv2d(x2, p[pre + "conv3.weight"], bf16=bf16), p, bufs, pre + "bn3.", BN_EPS_BLOCK, train)
    if res_conv:
        residual = rm(bn(conv2d(residual, p[pre + "residual_conv.weight"], stride=stride, bf16=bf16), p, bufs,
                         pre + "residual_bn.", BN_EPS_BLOCK, train))
    return rm(F.relu(x + residual)), x2


def block(p, pre, t, heads, bf16=False):
    """conformer.Block (code/models/conformer.py:55-72), rounding points as ref._trunk."""
    B, N, D = t.shape
    hd = D // heads
    r = _bf if bf16 else (lambda v: v)
    h = r(F.layer_norm(t, (D,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], LN_EPS_BLOCK))
    qkv = r(F.linear(h, r(p[pre + "attn.qkv.weight"]), p[pre + "attn.qkv.bias"]))
    qkv = qkv.reshape(B, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    attn = (q @ k.transpose(-2, -1)) * hd ** -0.5
    if bf16:
        e = torch.exp(attn - attn.amax(-1, keepdim=True))
        o = (_bf(e) @ v) / e.sum(-1, keepdim=True)
    else:
        o = attn.softmax(dim=-1) @ v
    o = r(o.transpose(1, 2).reshape(B, N, D))
    t = t + F.linear(o, r(p[pre + "attn.proj.weight"]), p[pre + "attn.proj.bias"])
    h = r(F.layer_norm(t, (D,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], LN_EPS_BLOCK))
    gelu = _GeluB16.apply if bf16 else F.gelu
    h = r(gelu(F.linear(h, r(p[pre + "mlp.fc1.weight"]), p[pre + "mlp.fc1.bias"])))
    return t + F.linear(h, r(p[pre + "mlp.fc2.weight"]), p[pre + "mlp.fc2.bias"])


def fcu_down(p, pre, x2, x_t, dw, bf16=False, maps=False):
    """FCUDown.forward (code/models/conformer.py:161-170).  maps: the device's order -- the bf16 map
    pooled (and stored bf16) before the 1x1 conv, which commutes with the pooling in exact arithmetic."""
    if maps:
        xp = _RoundMap.apply(F.avg_pool2d(x2, dw, dw)) if dw > 1 else x2
        x = conv2d(xp, p[pre + "conv_project.weight"], p[pre + "conv_project.bias"], bf16=bf16)
        x = x.flatten(2).transpose(1, 2)
    else:
        x = conv2d(x2, p[pre + "conv_project.weight"], p[pre + "conv_project.bias"], bf16=bf16)
        x = F.avg_pool2d(x, dw, dw).flatten(2).transpose(1, 2)
    x = F.gelu(F.layer_norm(x, (x.shape[-1],), p[pre + "ln.weight"], p[pre + "ln.bias"], LN_EPS_BLOCK))
    return torch.cat([x_t[:, 0][:, None, :], x], dim=1)


def fcu_up(p, bufs, pre, x_t, H, W, up, train=True, bf16=False, maps=False):
    """FCUUp.forward (code/models/conformer.py:187-194)."""
    rm, bn = (_RoundMap.apply, _bn_map) if maps else (_ident, _bn)
    B, _, C = x_t.shape
    x_r = x_t[:, 1:].transpose(1, 2).reshape(B, C, H, W)
    x_r = rm(F.relu(bn(conv2d(x_r, p[pre + "conv_project.weight"], p[pre + "conv_project.bias"], bf16=bf16), p, bufs,
                       pre + "bn.", BN_EPS_BLOCK, train)))
    return F.interpolate(x_r, size=(H * up, W * up))


def conformer_forward(p, bufs, x, cfg, train=True, bf16=False, bf16_conv=None, bf16_maps=False):
    """Conformer.forward (code/models/conformer.py:418-445) -> (conv_cls, trans_cls).  bf16_conv
    (default: bf16) selects the conv rounding points separately (the device's fp32-conv mode); bf16_maps
    the bf16 CNN maps (with bf16 convs only)."""
    B = x.shape[0]
    tb16, bf16 = bf16, bf16 if bf16_conv is None else bf16_conv
    maps = bool(bf16_maps and bf16)
    x_base = F.max_pool2d(F.relu(_bn(F.conv2d(x, p["conv1.weight"], stride=2, padding=3), p, bufs, "bn1.",
                                     BN_EPS_STEM, train)), 3, 2, 1)
    if maps:
        x_base = _RoundMap.apply(x_base)
    x, _ = conv_block(p, bufs, "conv_1.", x_base, 1, True, train=train, bf16=bf16, maps=maps)
    x_t = conv2d(x_base, p["trans_patch_conv.weight"], p["trans_patch_conv.bias"], stride=cfg.patch // 4, bf16=bf16)
    x_t = torch.cat([p["cls_token"].expand(B, -1, -1), x_t.flatten(2).transpose(1, 2)], dim=1)
    x_t = block(p, "trans_1.", x_t, cfg.heads, tb16)
    for name, _, _, res_conv, stride, dw, last in stages(cfg):
        pre = name + "."
        x, x2 = conv_block(p, bufs, pre + "cnn_block.", x, stride, res_conv, train=train, bf16=bf16, maps=maps)
        H, W = x2.shape[2:]
        x_st = fcu_down(p, pre + "squeeze_block.", x2, x_t, dw, bf16, maps)
        x_t = block(p, pre + "trans_block.", x_st + x_t, cfg.heads, tb16)
        x_t_r = fcu_up(p, bufs, pre + "expand_block.", x_t, H // dw, W // dw, dw, train, bf16, maps)
        x, _ = conv_block(p, bufs, pre + "fusion_block.", x, 2 if last else 1, last, x_t=x_t_r, train=train,
                          bf16=bf16, maps=maps)
    conv_cls = F.linear(F.adaptive_avg_pool2d(x, 1).flatten(1), p["conv_cls_head.weight"], p["conv_cls_head.bias"])
    x_t = F.layer_norm(x_t, (cfg.dim,), p["trans_norm.weight"], p["trans_norm.bias"], LN_EPS_TRANS_NORM)
    trans_cls = F.linear(x_t[:, 0], p["trans_cls_head.weight"], p["trans_cls_head.bias"])
    return conv_cls, trans_cls


def is_buffer(name):
    return name.endswith(("running_mean", "running_var", "num_batches_tracked"))


class SemiFormerRef:
    """One SSL step of SemiFormer.train_one (code/semiformer.py:103-146)."""

    def __init__(self, state, cfg, class_weights=None, thres=0.95, lambda_u=1.0, lr=1e-3, ema_decay=0.999,
                 bf16=False, bf16_conv=None, bf16_maps=False):
        self.cfg, self.bf16, self.bf16_conv, self.bf16_maps = cfg, bf16, bf16_conv, bf16_maps
        self.names = [k for k in state if not is_buffer(k)]
        self.p = {k: state[k].detach().clone().float().requires_grad_(True) for k in self.names}
        self.bufs = {k: state[k].detach().clone() for k in state if is_buffer(k)}
        self.ema = {k: v.detach().clone() for k, v in state.items()}
        self.cw, self.thres, self.lambda_u, self.decay = class_weights, thres, lambda_u, ema_decay
        self.opt = torch.optim.Adam([self.p[k] for k in self.names], lr=lr, betas=(0.9, 0.999), eps=1e-8,
                                    weight_decay=0)

    def step(self, x, y, uw, us):
        bs = x.shape[0]
        out_conv, out_trans = conformer_forward(self.p, self.bufs, torch.cat((x, uw, us)), self.cfg, True, self.bf16,
                                              self.bf16_conv, self.bf16_maps)
        w_conv, s_conv = out_conv[bs:].chunk(2)
        s_trans = out_trans[bs:].chunk(2)[1]
        lx = F.cross_entropy(out_conv[:bs], y, weight=self.cw) + F.cross_entropy(out_trans[:bs], y, weight=self.cw)
        lu_c, _, pl, mask = consistency(w_conv, s_conv, self.thres)
        lu_t, mask_mean, _, _ = consistency(w_conv, s_trans, self.thres)
        loss = lx + self.lambda_u * (lu_c + lu_t)
        self.opt.zero_grad()
        loss.backward()
        grads = {k: self.p[k].grad.detach().clone() for k in self.names}
        self.opt.step()
        state = {k: self.p[k].detach() for k in self.names}
        state.update(self.bufs)
        ema_update(self.ema, state, self.decay)
        return {"lx": lx.item(), "lu": (lu_c + lu_t).item(), "loss": loss.item(), "mask_mean": mask_mean.item(),
                "pseudo_label": pl, "mask": mask, "out_conv": out_conv.detach(), "out_trans": out_trans.detach(),
                "grads": grads}
