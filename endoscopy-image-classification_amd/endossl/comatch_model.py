"""ModelwEmb over the native ViT (CoMatch's model): `model(x) -> (logits, fts, z)`.

Reference: `ModelwEmb` (code/models/custom_model.py:147-213) with `build_head(in_fts, C,
is_complex=True)` (:107-120) and `head_emb` + `Normalize(2)` (:136-145,201-205).  The reference's
`ModelwEmb` cannot build a working ViT (its `backbone = Sequential(children[:-1])` drops the
cls-token / pos-embed logic); here `fts` is what a ViT backbone provides: the
final-LayerNorm CLS token, and the parameter names keep ModelwEmb's head indices
(fc.0 / fc.3 / fc.4, head_emb.0 / head_emb.2) after the timm trunk names.

The heads run as fp32 kernels (comatch.hip) on [n, D] rows -- 0.3 GFLOP per 1,408 images against
the trunk's 13 TFLOP; BatchNorm1d couples the rows, so the backward covers every image.
"""
import math
from copy import deepcopy

import torch
import torch.nn as nn

from . import _lib, dist
from ._lib import call, ptr
from .vit import NativeViT, ViTConfig

DROP_P = 0.2          # Dropout(0.2) in build_head (code/models/custom_model.py:113)
BN_MOMENTUM, BN_EPS = 0.1, 1e-5
LEAKY_SLOPE = 0.1     # LeakyReLU(negative_slope=0.1) (code/models/custom_model.py:202)


class EmbHeads:
    """Launch sequence of ModelwEmb's fc / head_emb on the features (forward, backward)."""

    def __init__(self, cfg, device):
        self.cfg, self.device = cfg, device
        self._bufs = {}

    def bufs(self, n):
        if n not in self._bufs:
            D, F, C, L = self.cfg.dim, self.cfg.dim // 4, self.cfg.num_classes, self.cfg.low_dim
            z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=self.device)  # noqa: E731
            self._bufs[n] = {
                "u": z(n, F), "xhat": z(n, F), "rstd": z(F), "y": z(n, F), "logits": z(n, C),
                "e": z(n, 3 * L), "v": z(n, L), "z": z(n, L), "norm": z(n),
                "dy": z(n, F), "du": z(n, F), "dv": z(n, L), "de": z(n, 3 * L), "dfts": z(n, D),
                "ws": z(n * max(F, C, 3 * L, L)), "keep": torch.ones(n, F, dtype=torch.uint8, device=self.device),
                "s1": z(F), "s2": z(F), "sb": z(2 * F), "sbl": z(2 * F)}
        return self._bufs[n]

    def forward(self, view, bn, fts, keep, train):
        """view(name) -> parameter view; bn = (running_mean, running_var, num_batches_tracked);
        keep: uint8 [n, D/4] dropout keep-mask (train only).  Returns (logits, z) buffer views."""
        cfg, s = self.cfg, _lib.stream()
        n, D = int(fts.shape[0]), cfg.dim
        F, C, L = D // 4, cfg.num_classes, cfg.low_dim
        b = self.bufs(n)
        kp = ptr(keep) if train else None
        call("es_dense_fwd", ptr(fts), D, ptr(view("fc.0.weight")), ptr(view("fc.0.bias")), ptr(b["u"]), F, n, D, F, 1,
             0.0, kp, 1.0 / (1.0 - DROP_P), s)
        world = dist.world_size()
        if train and world > 1:
            # SyncBatchNorm: batch statistics over every rank's rows (the one-process batch of the
            # reference); two all-reduces of F floats (sum, then the centred sum of squares)
            N = float(n * world)
            call("es_bn1d_sums", ptr(b["u"]), F, n, F, None, N, ptr(b["s1"]), s)
            dist.allreduce_inplace_(b["s1"])
            call("es_bn1d_sums", ptr(b["u"]), F, n, F, ptr(b["s1"]), N, ptr(b["s2"]), s)
            dist.allreduce_inplace_(b["s2"])
            call("es_bn1d_fwd_global", ptr(b["u"]), F, ptr(view("fc.3.weight")), ptr(view("fc.3.bias")), ptr(b["s1"]),
                 ptr(b["s2"]), N, ptr(bn[0]), ptr(bn[1]), ptr(bn[2]), BN_MOMENTUM, BN_EPS, ptr(b["y"]), F,
                 ptr(b["xhat"]), ptr(b["rstd"]), n, F, s)
        else:
            call("es_bn1d_fwd", ptr(b["u"]), F, ptr(view("fc.3.weight")), ptr(view("fc.3.bias")), ptr(bn[0]),
                 ptr(bn[1]), ptr(bn[2]) if train else None, BN_MOMENTUM, BN_EPS, 1 if train else 0, ptr(b["y"]), F,
                 ptr(b["xhat"]), ptr(b["rstd"]), n, F, s)
        call("es_dense_fwd", ptr(b["y"]), F, ptr(view("fc.4.weight")), ptr(view("fc.4.bias")), ptr(b["logits"]), C, n,
             F, C, 0, 0.0, None, 1.0, s)
        call("es_dense_fwd", ptr(fts), D, ptr(view("head_emb.0.weight")), ptr(view("head_emb.0.bias")), ptr(b["e"]),
             3 * L, n, D, 3 * L, 2, LEAKY_SLOPE, None, 1.0, s)
        call("es_dense_fwd", ptr(b["e"]), 3 * L, ptr(view("head_emb.2.weight")), ptr(view("head_emb.2.bias")),
             ptr(b["v"]), L, n, 3 * L, L, 0, 0.0, None, 1.0, s)
        call("es_l2norm_fwd", ptr(b["v"]), L, ptr(b["z"]), L, ptr(b["norm"]), n, L, s)
        return b["logits"], b["z"]

    def backward(self, view, gview, fts, keep, dlogits, dz):
        """dlogits [n, C], dz [n, L] -> head parameter grads (written through gview) and returns
        dfts [n, D].  Uses the activations of the last train forward."""
        cfg, s = self.cfg, _lib.stream()
        n, D = int(fts.shape[0]), cfg.dim
        F, C, L = D // 4, cfg.num_classes, cfg.low_dim
        b = self.bufs(n)
        ws = b["ws"]
        call("es_dense_bwd", ptr(dlogits), C, None, 0, 0, 0.0, None, 1.0, ptr(b["y"]), F, ptr(view("fc.4.weight")),
             ptr(b["dy"]), F, 0, ptr(gview("fc.4.weight")), ptr(gview("fc.4.bias")), n, F, C, ptr(ws), s)
        world = dist.world_size()
        if world > 1:  # SyncBatchNorm backward: the global means of dY and dY * xhat
            call("es_bn1d_bwd_sums", ptr(b["dy"]), F, ptr(b["xhat"]), n, F, ptr(b["sbl"]), s)
            b["sb"].copy_(b["sbl"])
            dist.allreduce_inplace_(b["sb"])
            call("es_bn1d_bwd_global", ptr(b["dy"]), F, ptr(b["xhat"]), ptr(b["rstd"]), ptr(view("fc.3.weight")),
                 ptr(b["sb"]), ptr(b["sbl"]), float(n * world), ptr(b["du"]), F, ptr(gview("fc.3.weight")),
                 ptr(gview("fc.3.bias")), n, F, s)
        else:
            call("es_bn1d_bwd", ptr(b["dy"]), F, ptr(b["xhat"]), ptr(b["rstd"]), ptr(view("fc.3.weight")), ptr(b["du"]),
                 F, ptr(gview("fc.3.weight")), ptr(gview("fc.3.bias")), n, F, s)
        call("es_dense_bwd", ptr(b["du"]), F, ptr(b["u"]), F, 1, 0.0, ptr(keep), 1.0 / (1.0 - DROP_P), ptr(fts), D,
             ptr(view("fc.0.weight")), ptr(b["dfts"]), D, 0, ptr(gview("fc.0.weight")), ptr(gview("fc.0.bias")), n, D,
             F, ptr(ws), s)
        call("es_l2norm_bwd", ptr(dz), L, ptr(b["z"]), L, ptr(b["norm"]), ptr(b["dv"]), L, n, L, s)
        call("es_dense_bwd", ptr(b["dv"]), L, None, 0, 0, 0.0, None, 1.0, ptr(b["e"]), 3 * L,
             ptr(view("head_emb.2.weight")), ptr(b["de"]), 3 * L, 0, ptr(gview("head_emb.2.weight")),
             ptr(gview("head_emb.2.bias")), n, 3 * L, L, ptr(ws), s)
        call("es_dense_bwd", ptr(b["de"]), 3 * L, ptr(b["e"]), 3 * L, 2, LEAKY_SLOPE, None, 1.0, ptr(fts), D,
             ptr(view("head_emb.0.weight")), ptr(b["dfts"]), D, 1, ptr(gview("head_emb.0.weight")),
             ptr(gview("head_emb.0.bias")), n, D, 3 * L, ptr(ws), s)
        return b["dfts"]


class _BN(nn.Module):
    """Holds BatchNorm1d's buffers under ModelwEmb's state_dict names (fc.3.running_mean, ...)."""


class _ViTEmbFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        ctx.module = module
        logits, fts, z = module._run(x, train=True)
        return logits.clone(), fts.clone(), z.clone()

    @staticmethod
    def backward(ctx, dlogits, dfts, dz):
        m = ctx.module
        C, L = m.cfg.num_classes, m.cfg.low_dim
        n = m._last_n
        dlogits = dlogits if dlogits is not None else torch.zeros(n, C, device=m.flat.device)
        dz = dz if dz is not None else torch.zeros(n, L, device=m.flat.device)
        g = m.backward_from(dlogits.float().contiguous(), dz.float().contiguous(),
                            None if dfts is None else dfts.float().contiguous())
        return (None, None) + tuple(m.engine().view(g, name).view(shape) for name, shape in m.layout)


class NativeViTEmb(NativeViT):
    """ModelwEmb (CoMatch model) over the native ViT trunk: forward(x) -> (logits, fts, z)."""

    def __init__(self, cfg=None, seed=None, **kw):
        cfg = cfg if cfg is not None else ViTConfig(head="emb", **kw)
        if cfg.head != "emb":
            raise ValueError("NativeViTEmb needs ViTConfig(head='emb')")
        super().__init__(cfg, seed=seed)
        self._init_bn_buffers(torch.device("cpu"))
        self._heads = None
        self.drop_seed = 0 if seed is None else int(seed)
        self._drop_counter = 0
        self._last_n = 0

    def _init_bn_buffers(self, device):
        F = self.cfg.dim // 4
        bn = self.fc._modules["3"]
        bn.register_buffer("running_mean", torch.zeros(F, device=device))
        bn.register_buffer("running_var", torch.ones(F, device=device))
        bn.register_buffer("num_batches_tracked", torch.zeros((), dtype=torch.int64, device=device))

    @property
    def fc(self):  # ModelwEmb.fc = the complex head (code/models/custom_model.py:196)
        return self._modules["fc"]

    @property
    def head_emb(self):
        return self._modules["head_emb"]

    def bn_buffers(self):
        bn = self.fc._modules["3"]
        return bn.running_mean, bn.running_var, bn.num_batches_tracked

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        bn = self.fc._modules["3"]
        for k in ("running_mean", "running_var", "num_batches_tracked"):
            bn._buffers[k] = fn(bn._buffers[k])
        self._heads = None
        return self

    def __deepcopy__(self, memo):
        other = NativeViTEmb.__new__(NativeViTEmb)
        nn.Module.__init__(other)
        other.cfg, other.layout, other.offs, other.numel = self.cfg, self.layout, self.offs, self.numel
        other._set_flat(self.flat.detach().clone())
        other._init_bn_buffers(self.flat.device)
        for a, b in zip(other.bn_buffers(), self.bn_buffers()):
            a.copy_(b)
        other._engine, other._heads = None, None
        other.precision = self.precision
        other.version = 0
        other.drop_seed, other._drop_counter, other._last_n = self.drop_seed, self._drop_counter, 0
        other.train(self.training)
        return other

    def heads(self):
        if self._heads is None or self._heads.device != self.flat.device:
            self._heads = EmbHeads(self.cfg, self.flat.device)
        return self._heads

    def dropout_keep(self, n):
        """Fresh Dropout(0.2) keep-mask for n rows (device hash, reproducible from drop_seed)."""
        keep = self.heads().bufs(n)["keep"]
        call("es_dropout_keep", ptr(keep), keep.numel(), DROP_P, self.drop_seed, self._drop_counter, _lib.stream())
        self._drop_counter += keep.numel()
        return keep

    def _run(self, images, train, keep=None, trunk_train=None):
        """Trunk features + heads.  images: tensor or list of tensors (one batch, no concat).
        trunk_train=False: the trunk in inference form (no saved activations; a frozen trunk)."""
        eng = self.engine()
        eng.pack(self.flat, self.version)
        imgs = images if isinstance(images, (list, tuple)) else [images]
        trunk_train = train if trunk_train is None else trunk_train
        self._last_trunk_train = trunk_train
        fts = eng.forward(self.flat, imgs, train=trunk_train)
        n = int(fts.shape[0])
        self._last_n = n
        if train and keep is None:
            keep = self.dropout_keep(n)
        self._last_keep = keep
        logits, z = self.heads().forward(lambda nm: eng.view(self.flat, nm), self.bn_buffers(), fts, keep, train)
        return logits, fts, z

    def backward_from(self, dlogits, dz, dfts_extra=None, grad_ready=None, trunk=True):
        """Gradient of the last train forward: dlogits [n, C], dz [n, L] (and optionally a direct
        dL/dfts) -> flat grad (returned).  grad_ready: Engine.backward's per-block hook.
        trunk=False (IS_FREEZE): the heads' parameter gradients only, the trunk's stay zero."""
        eng = self.engine()
        g = self.flat_grad
        g.zero_()
        fts = eng.acts(self._last_n, getattr(self, "_last_trunk_train", True)).fts
        dfts = self.heads().backward(lambda nm: eng.view(self.flat, nm), lambda nm: eng.view(g, nm), fts,
                                     self._last_keep, dlogits, dz)
        if dfts_extra is not None:
            dfts.add_(dfts_extra)
        if not trunk:
            return g
        return eng.backward(self.flat, g, dfts=dfts, zero_grad=False, grad_ready=grad_ready)

    def forward(self, x):
        if torch.is_grad_enabled() and self.training and any(p.requires_grad for p in self.parameters()):
            params = [self.get_parameter(name) for name, _ in self.layout]
            return _ViTEmbFunction.apply(x, self, *params)
        logits, fts, z = self._run(x, train=self.training)
        return logits.clone(), fts.clone(), z.clone()
