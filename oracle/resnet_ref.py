"""ORACLE (test infrastructure only): CPU fp32 restatement of timm's resnet18 and one step of the
reference's supervised trainer (BASELINE configs[0]).

  * resnet18                    timm==0.5.4 `resnet18` as `code/build.py:218-220` creates it (timm is
                                absent here: its published architecture is restated -- conv1 7x7/2,
                                BatchNorm(eps 1e-5), ReLU, max-pool 3/2/1, BasicBlocks [2, 2, 2, 2] at
                                64/128/256/512 channels with a 1x1/2 conv + BN shortcut where the shape
                                changes, global average pool, fc).  PARITY UNPINNED against timm
                                itself (no reference fixture holds a ResNet-18 output); the arithmetic
                                is torch's own conv / batch_norm / linear.
  * SupLearning step            code/supervised.py:111-138 (plain path): F.cross_entropy(weight=w,
                                reduction='mean') (`ce_loss` type 'none', code/loss.py:118), Adam(wd 0,
                                code/optimizer.py:13-53), EMA over every state entry (code/ema.py:51-59).
bf16=True applies the device's rounding points: the operands of every conv with both channel counts
multiples of 32 (conformer_ref.conv2d), i.e. all but the stem.  maps=True (with bf16) adds the device's
bf16 activation / gradient maps (resnet.NativeResNet.map_bf16), as conformer_ref's bf16_maps: the
max-pooled stem map, every BatchNorm (+ residual) (+ ReLU) output and the gradient arriving at each is
rounded to bf16; BatchNorms take their batch statistics from the conv's fp32 output.
"""
import torch
import torch.nn.functional as F

from .conformer_ref import _bn_map, _RoundMap, conv2d, is_buffer
from .ref import ema_update

BN_EPS = 1e-5


def blocks(layers=(2, 2, 2, 2), widths=(64, 128, 256, 512)):
    out, inp = [], 64
    for si, (n, w) in enumerate(zip(layers, widths)):
        for bi in range(n):
            stride = 2 if (si > 0 and bi == 0) else 1
            out.append((f"layer{si + 1}.{bi}.", inp, w, stride, stride != 1 or inp != w))
            inp = w
    return out


def _bn(x, p, bufs, pre, train):
    y = F.batch_norm(x, bufs[pre + "running_mean"], bufs[pre + "running_var"], p[pre + "weight"], p[pre + "bias"],
                     training=train, momentum=0.1, eps=BN_EPS)
    if train:
        bufs[pre + "num_batches_tracked"] += 1
    return y


def resnet18_forward(p, bufs, x, train=True, bf16=False, maps=False):
    """timm ResNet.forward (forward_features + global pool + fc); maps: the device's bf16 maps."""
    maps = bool(maps and bf16)
    if maps:
        rm = _RoundMap.apply

        def bn(y, pre):
            return _bn_map(y, p, bufs, pre, BN_EPS, train)
    else:
        def rm(v):
            return v

        def bn(y, pre):
            return _bn(y, p, bufs, pre, train)
    h = rm(F.max_pool2d(F.relu(_bn(F.conv2d(x, p["conv1.weight"], stride=2, padding=3), p, bufs, "bn1.", train)),
                        3, 2, 1))
    for pre, _, _, stride, ds in blocks():
        o = rm(F.relu(bn(conv2d(h, p[pre + "conv1.weight"], stride=stride, padding=1, bf16=bf16), pre + "bn1.")))
        o = bn(conv2d(o, p[pre + "conv2.weight"], padding=1, bf16=bf16), pre + "bn2.")
        sc = rm(bn(conv2d(h, p[pre + "downsample.0.weight"], stride=stride, bf16=bf16), pre + "downsample.1.")) \
            if ds else h
        h = rm(F.relu(o + sc))
    return F.linear(F.adaptive_avg_pool2d(h, 1).flatten(1), p["fc.weight"], p["fc.bias"])


class SupervisedRef:
    """One step of SupLearning.train_one's plain path (code/supervised.py:111-138)."""

    def __init__(self, state, class_weights=None, lr=1e-3, ema_decay=0.999, bf16=False):
        self.names = [k for k in state if not is_buffer(k)]
        self.p = {k: state[k].detach().clone().float().requires_grad_(True) for k in self.names}
        self.bufs = {k: state[k].detach().clone() for k in state if is_buffer(k)}
        self.ema = {k: v.detach().clone() for k, v in state.items()}
        self.cw, self.decay, self.bf16 = class_weights, ema_decay, bf16
        self.opt = torch.optim.Adam([self.p[k] for k in self.names], lr=lr, betas=(0.9, 0.999), eps=1e-8,
                                    weight_decay=0)

    def step(self, x, y):
        logits = resnet18_forward(self.p, self.bufs, x, True, self.bf16)
        loss = F.cross_entropy(logits, y, weight=self.cw, reduction="mean")
        self.opt.zero_grad()
        loss.backward()
        grads = {k: self.p[k].grad.detach().clone() for k in self.names}
        self.opt.step()
        state = {k: self.p[k].detach() for k in self.names}
        state.update(self.bufs)
        ema_update(self.ema, state, self.decay)
        return {"loss": loss.item(), "logits": logits.detach(), "grads": grads}
