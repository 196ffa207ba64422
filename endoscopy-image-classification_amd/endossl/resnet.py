"""Native ResNet-18 -- the supervised baseline of BASELINE configs[0] (SURVEY.md §8(d) P0:
`supervised.py` ResNet-18, 23 classes, B=16, 224²) on the Conformer's CNN kernels.

Reference: `build_model` -> timm `resnet18` (`code/build.py:160-211`, timm==0.5.4, absent from this
image: its architecture is restated here -- conv1 7x7/2 -> BatchNorm -> ReLU -> max-pool 3/2 -> four
stages of two BasicBlocks (3x3 conv -> BN -> ReLU -> 3x3 conv -> BN, + identity or 1x1/2 conv + BN
shortcut, ReLU) -> global average pool -> fc).  `model(x) -> logits`, the timm state_dict (names
and order), so checkpoints interchange.

MI355X layout (as NativeConformer, whose parameter plumbing it shares): parameters in one flat fp32
buffer, NHWC maps, every conv an implicit GEMM (bf16 operands for channel counts % 32 == 0 --
all but the 3-channel stem; `set_conv_precision("fp32")` for parity), BatchNorm with the residual add
and ReLU fused into its apply pass, SyncBatchNorm at N > 1 (as the Conformer).  With the bf16 convs
the activation and gradient maps after the stem's max-pool are bf16 (map_bf16; the stem and BatchNorm
statistics stay fp32, ENDOSSL_MAP_BF16=0 keeps fp32 maps): every conv after the stem is bf16-eligible.
"""
import math

import torch
import torch.nn as nn

from . import _lib
from .conformer import (BN_EPS_STEM, CONV_BF16, GRAD_SINKS, MAP_BF16, NativeConformer, _ConvHeadFn, _GradSink, _Map,
                        _map_dtype, _MaxPoolFn, _join_queued, _rup, bn, bn_conv, conv)

BN_EPS = 1e-5  # timm BasicBlock norm_layer = nn.BatchNorm2d (default eps)


class ResNetConfig:
    def __init__(self, layers=(2, 2, 2, 2), num_classes=23, img_size=224, widths=(64, 128, 256, 512)):
        self.layers, self.widths = tuple(layers), tuple(widths)
        self.num_classes, self.img_size = num_classes, img_size

    def blocks(self):
        """(prefix, inplanes, planes, stride, downsample) per BasicBlock in state_dict order."""
        out, inp = [], 64
        for si, (n, w) in enumerate(zip(self.layers, self.widths)):
            for bi in range(n):
                stride = 2 if (si > 0 and bi == 0) else 1
                out.append((f"layer{si + 1}.{bi}.", inp, w, stride, stride != 1 or inp != w))
                inp = w
        return out


def _bn_entries(pre, C):
    return [(pre + "weight", (C,), "p"), (pre + "bias", (C,), "p"), (pre + "running_mean", (C,), "rm"),
            (pre + "running_var", (C,), "rv"), (pre + "num_batches_tracked", (), "nbt")]


def resnet_layout(cfg):
    """(name, shape, kind) in timm resnet18's state_dict order."""
    out = [("conv1.weight", (64, 3, 7, 7), "p")] + _bn_entries("bn1.", 64)
    for pre, inp, w, stride, ds in cfg.blocks():
        out += [(pre + "conv1.weight", (w, inp, 3, 3), "p")] + _bn_entries(pre + "bn1.", w)
        out += [(pre + "conv2.weight", (w, w, 3, 3), "p")] + _bn_entries(pre + "bn2.", w)
        if ds:
            out += [(pre + "downsample.0.weight", (w, inp, 1, 1), "p")] + _bn_entries(pre + "downsample.1.", w)
    C = cfg.num_classes
    out += [("fc.weight", (C, cfg.widths[-1]), "p"), ("fc.bias", (C,), "p")]
    return out


def init_resnet_(flat, layout, offs, generator=None):
    """timm ResNet.init_weights: kaiming-normal (fan_out, ReLU) convs, BatchNorm weight 1 / bias 0,
    fc as nn.Linear's default (uniform +-1/sqrt(fan_in) for weight and bias)."""
    for name, shape, kind in layout:
        if kind != "p":
            continue
        t = flat[offs[name]:offs[name] + math.prod(shape)].view(shape)
        if len(shape) == 4:
            std = math.sqrt(2.0 / (shape[0] * shape[2] * shape[3]))
            t.normal_(0.0, std, generator=generator)
        elif name.startswith("fc."):
            bound = 1.0 / math.sqrt(layout[-2][1][1])
            t.uniform_(-bound, bound, generator=generator)
        elif name.endswith("weight"):
            t.fill_(1.0)
        else:
            t.zero_()


class NativeResNet(NativeConformer):
    """ResNet-18 whose compute runs in libendossl_hip.so; state_dict identical to timm's resnet18.
    Shares NativeConformer's flat-parameter plumbing (views, BatchNorm buffers, bf16 conv images,
    device moves, deepcopy) and its conv / BatchNorm / pooling / head autograd Functions."""

    def __init__(self, cfg=None, seed=None, **kw):
        nn.Module.__init__(self)
        self.cfg = cfg if cfg is not None else ResNetConfig(**kw)
        self.layout = resnet_layout(self.cfg)
        self.offs, o = {}, 0
        for name, shape, kind in self.layout:
            if kind == "p":
                self.offs[name] = o
                o = _rup(o + math.prod(shape), 64)
        self.numel = o
        self.shapes = {name: shape for name, shape, _ in self.layout}
        flat = torch.zeros(self.numel, dtype=torch.float32)
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        init_resnet_(flat, self.layout, self.offs, generator=gen)
        self._build(flat, device=torch.device("cpu"))
        self.version = 0
        self.cur_n = 0
        self.conv_bf16 = CONV_BF16

    @property
    def map_bf16(self):
        """bf16 activation / gradient maps after the stem's max-pool (every later conv has channel counts
        % 32 == 0, so all of them run on the bf16 kernels)."""
        return bool(self.conv_bf16 and MAP_BF16)

    @property
    def fc(self):  # a real submodule here (timm's classifier, IS_FREEZE's trainable part)
        return self._modules["fc"]

    def no_weight_decay(self):
        return set()

    def _pack(self):  # no transformer weight images
        return None

    def _block(self, x, pre, inp, planes, stride, ds):
        """timm BasicBlock.forward: relu(bn2(conv2(relu(bn1(conv1(x))))) + shortcut)."""
        sink = _GradSink() if GRAD_SINKS else None  # x's two gradient contributions summed in place
        h = conv(self, x, _Map.nhwc(x), pre + "conv1.weight", None, planes, 3, stride, 1, stats=True, sink=sink)
        # bn1 + ReLU feed conv2 alone: applied by conv2's gathers where the bf16 kernels run it (bn_conv)
        h = bn_conv(self, h, pre + "bn1.", pre + "conv2.weight", None, planes, 3, 1, 1, stats=True, eps=BN_EPS)
        if ds:
            sc = conv(self, x, _Map.nhwc(x), pre + "downsample.0.weight", None, planes, 1, stride, 0, stats=True,
                      sink=sink)
            sc = bn(self, sc, pre + "downsample.1.", eps=BN_EPS)
            return bn(self, h, pre + "bn2.", eps=BN_EPS, relu=True, res=sc)
        return bn(self, h, pre + "bn2.", eps=BN_EPS, relu=True, res=x, res_sink=sink)

    def forward(self, x):
        cfg = self.cfg
        if not self.flat.is_cuda:
            raise _lib.EndosslCallError("NativeResNet runs on the MI355X only: move it to a cuda device first")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected [n, 3, H, W] images, got {tuple(x.shape)}")
        _join_queued.clear()
        self._bn_partials.clear()
        n, H, W = x.shape[0], x.shape[2], x.shape[3]
        self.cur_n = n
        x = x.float().permute(0, 2, 3, 1).contiguous()  # NHWC once (the stem's 3-channel gathers)
        img = _Map(x, n, H, W, 3, sn=3 * H * W, sh=3 * W, sw=3, sc=1)
        on_tape = torch.is_grad_enabled() and self.training
        frozen = getattr(self, "frozen_trunk", False)
        anchor = self._anchor if (on_tape and not frozen) else None
        h = conv(self, x, img, "conv1.weight", None, 64, 7, 2, 3, anchor=anchor, out_dtype=torch.float32)
        h = _MaxPoolFn.apply(bn(self, h, "bn1.", eps=BN_EPS_STEM, relu=True), 3, 2, 1, _map_dtype(self))
        for pre, inp, planes, stride, ds in cfg.blocks():
            h = self._block(h, pre, inp, planes, stride, ds)
        head_anchor = self._anchor if (on_tape and frozen) else None
        return _ConvHeadFn.apply(h, self, head_anchor, "fc.")
