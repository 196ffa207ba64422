"""Native ViT backbone for the SSL step: timm-0.5.4 layout, MI355X kernels underneath.

Reference: `build.build_model` -> `timm.create_model('vit_small_patch16_224', num_classes=C)`
(code/build.py:196-197); block arithmetic pinned by code/models/conformer.py:8-72 (Mlp,
Attention, Block: LN eps 1e-6, qkv_bias, scale hd^-0.5, exact GELU); wrapper = timm
VisionTransformer (PatchEmbed Conv2d(3,D,16,16) -> cat CLS -> + pos_embed -> blocks -> norm ->
head on CLS, as in code/models/conformer.py:420,430,442-443).

MI355X-first layout:
  * every parameter lives in ONE fp32 flat buffer (`flat`), state_dict names/order identical to
    timm (checkpoints interchange); grads, Adam moments and the EMA are flat buffers of the same
    layout, so the optimizer + EMA is a single HBM sweep (optim.hip);
  * the GEMMs read bf16 weight images W [N,K] and W^T [K,N] that the optimizer step re-packs;
  * activations are token-major [tokens, features], padded to 256 rows (zero pad), fp32 for the
    residual stream, bf16 for GEMM operands;
  * forward / backward are explicit sequences of C-ABI launches on the current stream (no
    autograd graph on the hot path); `NativeViT.forward` wraps them in one autograd.Function so
    `model(x)` / `loss.backward()` still work as a drop-in nn.Module.
"""
import ctypes
import math
import os

import torch
import torch.nn as nn

from . import _lib
from ._lib import call, ptr

EPI_BF16, EPI_GELU, EPI_F32_RESID, EPI_DGELU, EPI_F32, EPI_PATCH, EPI_GELU_ACT, EPI_GELU_D, EPI_MULAUX = range(9)
# LayerNorm backward workgroups (grid-stride over row pairs; per-workgroup dgamma / dbeta partials)
LN_BWD_BLOCKS = 1024
# HIP priority of the second stream (weak forward, overlapped weight gradients) for steps of at least
# SIDE_PRIORITY_MIN_M train tokens (below it: 0, the default stream's).  Same-box A/Bs (profiles/r04_stream_priority.txt,
# DESIGN.md §5): F1 (100,864 tokens) -1 vs 0 30.34 / 30.33 / 30.22 vs
# 30.59 / 30.51 / 30.39 ms; the N = 8 shard (12,608) 5.35 / 5.36 vs 5.32 / 5.31
SIDE_PRIORITY = -1
SIDE_PRIORITY_MIN_M = 65536


# code/dataset.py:21-22 (transforms.Normalize on every ViT input); uint8 batches are normalised on the GPU
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _rup(x, m):
    return (x + m - 1) // m * m


class ViTConfig:
    """head = "cls": timm's Linear head on the CLS token (FixMatch / SemiFormer-style models);
    head = "emb": ModelwEmb's heads on the final-LN CLS feature (CoMatch, code/models/custom_model.py:
    147-213): fc = Linear(D, D/4) -> ReLU -> Dropout(0.2) -> BatchNorm1d -> Linear(D/4, C) and
    head_emb = Linear(D, 3L) -> LeakyReLU(0.1) -> Linear(3L, L) -> Normalize(2), L = low_dim."""

    def __init__(self, img_size=224, patch=16, dim=384, depth=12, heads=6, mlp_ratio=4.0, num_classes=23,
                 eps=1e-6, head="cls", low_dim=64):
        self.img_size, self.patch, self.dim, self.depth = img_size, patch, dim, depth
        self.heads, self.num_classes, self.eps = heads, num_classes, eps
        self.head, self.low_dim = head, low_dim
        assert head in ("cls", "emb")
        self.hidden = int(dim * mlp_ratio)
        self.grid = img_size // patch
        self.np = self.grid * self.grid
        self.T = self.np + 1
        assert dim == heads * 64, "kernels assume head_dim 64"
        assert dim % 128 == 0 and self.hidden % 128 == 0

    def as_dict(self):
        return dict(img_size=self.img_size, patch=self.patch, dim=self.dim, depth=self.depth, heads=self.heads,
                    mlp_ratio=self.hidden / self.dim, num_classes=self.num_classes, eps=self.eps, head=self.head,
                    low_dim=self.low_dim)


VIT_CONFIGS = {
    "vit_small_patch16_224": dict(img_size=224, dim=384, depth=12, heads=6),
    "vit_small_patch16_384": dict(img_size=384, dim=384, depth=12, heads=6),
    "vit_base_patch16_224": dict(img_size=224, dim=768, depth=12, heads=12),
    "vit_tiny_test": dict(img_size=64, dim=128, depth=2, heads=2),
}


def emb_head_layout(cfg):
    """ModelwEmb heads (code/models/custom_model.py:110-116 build_head(is_complex=True) indices
    0 Linear, 3 BatchNorm1d, 4 Linear; :201-205 head_emb indices 0 Linear, 2 Linear)."""
    D, C, L, F = cfg.dim, cfg.num_classes, cfg.low_dim, cfg.dim // 4
    return [("fc.0.weight", (F, D)), ("fc.0.bias", (F,)), ("fc.3.weight", (F,)), ("fc.3.bias", (F,)),
            ("fc.4.weight", (C, F)), ("fc.4.bias", (C,)), ("head_emb.0.weight", (3 * L, D)),
            ("head_emb.0.bias", (3 * L,)), ("head_emb.2.weight", (L, 3 * L)), ("head_emb.2.bias", (L,))]


def param_layout(cfg):
    """timm 0.5.4 VisionTransformer state_dict order: (name, shape); the "emb" head replaces
    `head` with ModelwEmb's fc / head_emb parameters."""
    D, Hd, C = cfg.dim, cfg.hidden, cfg.num_classes
    out = [("cls_token", (1, 1, D)), ("pos_embed", (1, cfg.T, D)),
           ("patch_embed.proj.weight", (D, 3, cfg.patch, cfg.patch)), ("patch_embed.proj.bias", (D,))]
    for i in range(cfg.depth):
        b = f"blocks.{i}."
        out += [(b + "norm1.weight", (D,)), (b + "norm1.bias", (D,)),
                (b + "attn.qkv.weight", (3 * D, D)), (b + "attn.qkv.bias", (3 * D,)),
                (b + "attn.proj.weight", (D, D)), (b + "attn.proj.bias", (D,)),
                (b + "norm2.weight", (D,)), (b + "norm2.bias", (D,)),
                (b + "mlp.fc1.weight", (Hd, D)), (b + "mlp.fc1.bias", (Hd,)),
                (b + "mlp.fc2.weight", (D, Hd)), (b + "mlp.fc2.bias", (D,))]
    out += [("norm.weight", (D,)), ("norm.bias", (D,))]
    if cfg.head == "emb":
        out += emb_head_layout(cfg)
    else:
        out += [("head.weight", (C, D)), ("head.bias", (C,))]
    offs, o = {}, 0
    for name, shape in out:
        offs[name] = o
        o = _rup(o + math.prod(shape), 64)  # 256-B aligned tensors (16-B vector access everywhere)
    return out, offs, o


def timm_init_(flat, cfg, layout, offs, generator=None):
    """timm 0.5.4 `_init_vit_weights` (jax_impl=False): Linear trunc_normal(.02)/zero bias, head
    zero, LayerNorm ones/zeros, pos_embed & cls_token trunc_normal(.02); patch conv keeps the
    PyTorch Conv2d default (kaiming_uniform a=sqrt(5)).  Parity unpinned (timm absent here)."""
    with torch.no_grad():
        flat.zero_()
        for name, shape in layout:
            t = flat[offs[name]:offs[name] + math.prod(shape)].view(shape)
            if name in ("cls_token", "pos_embed"):
                nn.init.trunc_normal_(t, std=0.02, generator=generator)
            elif name == "patch_embed.proj.weight":
                nn.init.kaiming_uniform_(t, a=math.sqrt(5), generator=generator)
            elif name == "patch_embed.proj.bias":
                bound = 1.0 / math.sqrt(3 * cfg.patch * cfg.patch)
                nn.init.uniform_(t, -bound, bound, generator=generator)
            elif name.startswith(("fc.", "head_emb.")):
                # ModelwEmb heads keep the PyTorch defaults: Linear kaiming_uniform(a=sqrt(5)) with
                # bias U(+-1/sqrt(fan_in)), BatchNorm1d weight 1 / bias 0
                if name == "fc.3.weight":
                    t.fill_(1.0)
                elif name == "fc.3.bias":
                    t.zero_()
                elif len(shape) == 2:
                    nn.init.kaiming_uniform_(t, a=math.sqrt(5), generator=generator)
                else:
                    w = [sh for nm, sh in layout if nm == name[:-len("bias")] + "weight"][0]
                    bound = 1.0 / math.sqrt(w[1])
                    nn.init.uniform_(t, -bound, bound, generator=generator)
            elif name.startswith("head"):
                t.zero_()
            elif name.endswith("weight") and len(shape) == 2:
                nn.init.trunc_normal_(t, std=0.02, generator=generator)
            elif "norm" in name and name.endswith("weight"):
                t.fill_(1.0)
            else:
                t.zero_()


class _Acts:
    """Token-major activation buffers for one batch size (train keeps every layer's tensors)."""

    def __init__(self, cfg, n, train, device, b16=torch.bfloat16):
        D, Hd, L = cfg.dim, cfg.hidden, cfg.depth
        self.n, self.train = n, train
        self.M = n * cfg.T
        # 256 rows beyond the padded token count: a half-batch lane's GEMM tiles (Engine.SHARD_LANES) start at
        # an image boundary and read up to 256 rows past their last token
        Mp = _rup(self.M, 256) + 256
        self.Mp = Mp
        Lk = L if train else 1
        f32 = torch.float32
        z = lambda *s, dt=f32: torch.zeros(*s, dtype=dt, device=device)  # noqa: E731
        self.patches = z(_rup(n * cfg.np, 256), 3 * cfg.patch * cfg.patch, dt=b16)
        self.x = z(L + 1 if train else 2, Mp, D)
        self.xmid = z(Lk, Mp, D)
        self.h1 = z(Lk, Mp, D, dt=b16)
        self.h2 = z(Lk, Mp, D, dt=b16)
        self.mean1, self.rstd1 = z(Lk, Mp), z(Lk, Mp)
        self.mean2, self.rstd2 = z(Lk, Mp), z(Lk, Mp)
        self.qkv = z(Lk, Mp, 3 * D, dt=b16)
        self.o = z(Lk, Mp, D, dt=b16)
        self.lse = z(Lk, n * cfg.heads * cfg.T)
        self.pre = z(Lk if train else 0, Mp, Hd, dt=b16)  # fc1 pre-activation, or its GELU' (Engine.GELU_D)
        self.act = z(Lk, Mp, Hd, dt=b16)
        # the last block on its CLS rows only (Engine.PRUNE_LAST): compact [n, .] images, rows padded to 256
        Mc = _rup(n, 256)
        self.c_o, self.c_lse = z(Mc, D, dt=b16), z(n * cfg.heads)
        self.c_h1 = z(Mc, D, dt=b16)  # LN1 output of the CLS rows (the last block's Q projection input)
        self.c_xmid, self.c_h2 = z(Mc, D), z(Mc, D, dt=b16)
        self.c_mean2, self.c_rstd2 = z(Mc), z(Mc)
        self.c_pre = z(Mc, Hd, dt=b16) if train else None
        self.c_act, self.c_xout = z(Mc, Hd, dt=b16), z(Mc, D)
        self.xhat = z(n, D)
        self.rstd_cls = z(n)
        self.logits = z(n, cfg.num_classes)
        self.fts = z(n, D) if cfg.head == "emb" else None


class _Grads:
    """Backward scratch (one layer's worth, reused top-down)."""

    def __init__(self, cfg, n, device, b16=torch.bfloat16):
        D, Hd = cfg.dim, cfg.hidden
        Mp = _rup(n * cfg.T, 256) + 256  # (+ 256: the half-batch lanes' tile over-read, as _Acts)
        f32 = torch.float32
        z = lambda *s, dt=f32: torch.zeros(*s, dtype=dt, device=device)  # noqa: E731
        self.n = n
        self.dx, self.dxb = z(Mp, D), z(Mp, D, dt=b16)
        self.dxm, self.dxmb = z(Mp, D), z(Mp, D, dt=b16)
        self.dh = z(Mp, D, dt=b16) if Engine.DH_BF16 else z(Mp, D)  # d(LN output) from the dgrad GEMMs
        self.dpre = z(Mp, Hd, dt=b16)
        self.dqkv = z(Mp, 3 * D, dt=b16)
        self.do = z(Mp, D, dt=b16)
        self.dpatch = z(_rup(n * cfg.np, 256), D, dt=b16)
        self.dyn = z(n, D)
        self.delta = z(n * cfg.heads * cfg.T)
        # last block on CLS rows (Engine.PRUNE_LAST): compact gradients, and d(xmid) as a full token
        # image whose non-CLS rows stay zero (only CLS rows are ever written)
        Mc = _rup(n, 256)
        self.c_dx, self.c_dxb = z(Mc, D), z(Mc, D, dt=b16)
        self.c_dpre, self.c_dxmb, self.c_do = z(Mc, Hd, dt=b16), z(Mc, D, dt=b16), z(Mc, D, dt=b16)
        self.c_dh = z(Mc, D, dt=b16) if Engine.DH_BF16 else z(Mc, D)
        self.dxm_cls = z(Mp, D)


class _TNProblem(ctypes.Structure):
    """es_tn_problem (include/endossl.h): one GEMM of a grouped weight-gradient launch."""
    _fields_ = [("dy", ctypes.c_void_p), ("x", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("bias_out", ctypes.c_void_p), ("M", ctypes.c_int), ("N1", ctypes.c_int), ("N2", ctypes.c_int),
                ("ld1", ctypes.c_int), ("ld2", ctypes.c_int), ("mchunk", ctypes.c_int), ("tile0", ctypes.c_int),
                ("pad", ctypes.c_int)]


class Engine:
    """Explicit forward / backward of the ViT over C-ABI kernels.  One per (model, device)."""

    # Kernel-choice and overlap settings.  Class attributes (tests override them per instance); the
    # measured A/Bs behind each value are in DESIGN.md §5.  Paths measured slower were removed in round 4
    # (two-lane backward, fused inference MLP, split attention backward): their record stays in DESIGN.md.
    #
    # split-K sizing of the weight-gradient GEMMs: floor(TN_TARGET_BLOCKS / tiles) splits, so the grid
    # never exceeds the target (768 leaves the data-gradient chain on the other stream room: 35.10-35.13
    # ms/step vs 35.41-35.43 at 1024, 35.99 at 512, r01).
    TN_TARGET_BLOCKS = 768
    # share of the CUs the overlapped long-axis weight-gradient launches are sized to (half: the 384 x 192
    # tile's 147-KiB workgroups otherwise hold every CU's LDS; F1 34.43 / 34.36 -> 33.66 / 33.84 ms, r02)
    TN_SHARE = 0.5
    TN_SHARE_MIN_M = 16384  # shortest token axis it applies to
    TN_MAX_SPLITS = 128
    # Weight gradients of a small shard (strong scaling: M = 12,608 train tokens per rank at N = 8) as ONE
    # grouped launch per GROUP_LAYERS layers after the data-gradient chain (es_gemm_tn_grouped: every
    # 128x128 tile over its GEMM's whole token axis -- no split-K slabs): B=8 6.11-6.15 vs 6.35 ms/step.
    # "auto": when the train tokens M < GROUP_WGRAD_MAX_M; "1" always; "0" never.  bf16 engines only.
    GROUP_WGRAD = "auto"
    GROUP_WGRAD_MAX_M = 16384
    GROUP_LAYERS = 6
    # ... and the data-gradient chain of blocks depth-2..0 as TWO lanes, the train images' halves on the caller's
    # stream and the side stream, the grouped weight gradients on a third stream after both lanes.  The second
    # stream is worth 13 % at N = 8 (6.25 -> 5.41 ms, weak forward / weight gradients beside the chain), but the
    # split chain measured slower: 5.35 / 5.35 / 5.44 vs 5.30 / 5.29 / 5.29 ms (r05, one box, interleaved; the
    # half-batch kernels lose more than the concurrency gains).  Off; bit-identical when on (test_gpu_step.py).
    SHARD_LANES = False
    # the LayerNorm backwards' parameter-gradient reductions off the data-gradient chain: each backward leaves its
    # per-workgroup partials in a workspace of its own and one es_ln_param_grads_multi launch per weight-gradient
    # launch reduces them on the side stream (24 launches fewer on the chain per step; bit-identical)
    DEFER_LN_GRADS = True
    LN_MULTI_MAX = 32  # entries per es_ln_param_grads_multi launch (RPM_MAX in csrc/gemm.hip)
    # A block's long-axis weight gradients (fc2, fc1, proj, qkv: 24 tiles of 384 x 192 at ViT-S) as ONE
    # split-K launch on the side stream once the block's data-gradient chain has produced its last dY
    # (es_gemm_tn_big_grouped) plus one reduce launch, sized to LAYER_TN_SHARE of the CUs (4 splits):
    # F1 31.53 -> 31.0 ms, C1 67.2 -> 66.8 (r03).
    LAYER_WGRAD = True
    LAYER_TN_SHARE = 0.375
    # second HIP stream: the weak forward beside the train forward ("fwd") and the weight-gradient
    # GEMMs beside the data-gradient chain ("bwd"); ENDOSSL_OVERLAP=0 serialises everything on the
    # caller's stream (a diagnostic: step_timeline / single-stream kernel tables)
    _OV = os.environ.get("ENDOSSL_OVERLAP", "1")
    OVERLAP_FWD = _OV in ("1", "fwd")
    OVERLAP = _OV in ("1", "bwd")
    # d(LN output) from the fc1 / qkv dgrad GEMMs in bf16 -- every GEMM operand of the backward is bf16
    # already; halves those epilogues' writes and the LN-backward reads
    DH_BF16 = True
    # the train fc1 forward stores GELU'(pre) instead of the pre-activation (EPI_GELU_D: shares the
    # erf's exp), so the fc2 dgrad epilogue is one multiply instead of an erf + two exps per element
    # (EPI_MULAUX)
    GELU_D = True
    # the last block on its CLS rows only: timm's head reads x[:, 0] after the last block
    # (VisionTransformer.forward_features / forward_head), so the last block's attention is needed for
    # the CLS queries only (over all keys) and its projection, LayerNorm 2 and MLP for the CLS rows
    # only; in the backward d(loss)/d(non-CLS rows) of the last block's output is exactly zero, so the
    # skipped rows contribute exactly nothing to any gradient.  False runs every row (tests compare).
    PRUNE_LAST = True
    # ... and its Q projection (forward) and Q weight gradient on the CLS rows only (False: all rows,
    # with a dQ that is zero off the CLS rows)
    PRUNE_Q = True
    # the attention projection, its residual add and LayerNorm 2 as one launch at D = 384 for token axes of at
    # least RESID_LN_MIN_M rows (es_gemm_nt_resid_ln: x is not re-read for its statistics; the same bits as the
    # two launches, tested).  Isolated (scripts/resid_ln_bench.py) 138 -> 108 us at F1's train rows, 121 -> 90 at
    # the weak rows, 58 -> 56 at a rank's share at N = 2, slower below (one persistent workgroup per CU with
    # 1.5-3 tiles each); F1 30.09 / 30.06 / 30.10 -> 29.85 / 29.90 / 29.86 ms and, on a second box, 30.38 / 30.40 /
    # 30.40 -> 30.22 / 30.21 / 30.21 (same box each, interleaved, scripts/gpu_ab_residln.sh).  ENDOSSL_RESID_LN=0
    # turns it off.
    RESID_LN = os.environ.get("ENDOSSL_RESID_LN", "1") == "1"
    RESID_LN_MIN_M = 40000

    # fp32 parity mode (csrc/parity.hip): the same launch sequence over fp32 operand storage; the
    # entry points with an fp32 form, by their bf16 names
    PARITY_NAMES = {n: n + "_f32" for n in (
        "es_gemm_nt", "es_gemm_tn", "es_attn_fwd", "es_attn_bwd", "es_attn_cls_fwd", "es_attn_cls_bwd",
        "es_layernorm_fwd", "es_layernorm_bwd", "es_patch_im2col", "es_patch_im2col_u8", "es_embed_bwd",
        "es_pack_weights")}
    PARITY_NAMES.update({"es_layernorm_bwd_b16": "es_layernorm_bwd_f32", "es_cast_f32_bf16": "es_copy_f32"})

    def __init__(self, cfg, device, precision="bf16"):
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be 'bf16' (production) or 'fp32' (parity mode), got {precision!r}")
        self.cfg, self.device = cfg, device
        self.precision = precision
        self.op_dtype = torch.bfloat16 if precision == "bf16" else torch.float32
        self.layout, self.offs, self.numel = param_layout(cfg)
        self.shapes = dict(self.layout)
        self._acts = {}
        self._grads = {}
        self._ws = None
        self._ws_ln = None
        self._ws_lnp = None
        self._lnp_next = 0
        self._side = None
        self._ncu = None
        self._lane_state = {}
        self._grad_b = None
        self.overlap = self.OVERLAP
        self.overlap_fwd = self.OVERLAP_FWD
        self._packed_version = -1
        D, Hd = cfg.dim, cfg.hidden
        b16 = self.op_dtype
        # bf16 weight images: W [N,K] for forward, W^T [K,N] for dgrad
        mats = [("patch_embed.proj.weight", D, 3 * cfg.patch * cfg.patch, False)]
        for i in range(cfg.depth):
            b = f"blocks.{i}."
            mats += [(b + "attn.qkv.weight", 3 * D, D, True), (b + "attn.proj.weight", D, D, True),
                     (b + "mlp.fc1.weight", Hd, D, True), (b + "mlp.fc2.weight", D, Hd, True)]
        self.wb, self.wt = {}, {}
        esz = _lib.load().es_pack_entry_size()
        raw = bytearray(esz * len(mats))
        for j, (name, N, K, need_t) in enumerate(mats):
            self.wb[name] = torch.zeros(N, K, dtype=b16, device=device)
            if need_t:
                self.wt[name] = torch.zeros(K, N, dtype=b16, device=device)
            dst_t = self.wt[name].data_ptr() if need_t else 0
            entry = (ctypes.c_long(self.offs[name]), ctypes.c_void_p(self.wb[name].data_ptr()),
                     ctypes.c_void_p(dst_t), ctypes.c_int(N), ctypes.c_int(K))
            buf = b"".join(bytes(e) for e in entry)
            raw[j * esz:j * esz + len(buf)] = buf
        self._pack_tab = torch.frombuffer(raw, dtype=torch.uint8).to(device)
        self._nmat = len(mats)
        # optional live timing of one launch site: {"label": str, "events": [(start, end, flops)]}
        self.probe = None
        # optional test hook (tests/test_gpu_blocks.py, teacher-forced per-block parity): called as
        # capture(kind, train, layer, *tensors) on the launch stream with the engine's own buffers --
        # "fwd" (block input, block output), "fwd_cls" (input, compact CLS-row output of the pruned last
        # block), "dtop" (d loss / d final-block output: compact CLS rows or full token rows), "bwd"
        # (d loss / d block input, after the block's reverse pass); the callee clones what it keeps
        self.capture = None

    def _call(self, name, *args):
        """C-ABI call; in parity mode the fp32 form of the entry point."""
        if self.precision == "fp32":
            name = self.PARITY_NAMES.get(name, name)
        return call(name, *args)

    def _gemm(self, label, *args):
        """es_gemm_nt, optionally bracketed by HIP events on the launch stream (bench roofline)."""
        pr = self.probe
        if pr is not None and pr["label"] == label:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self._call("es_gemm_nt", *args)
            e1.record()
            M, N, K = args[11], args[12], args[13]
            pr["events"].append((e0, e1, 2.0 * M * N * K))
        else:
            self._call("es_gemm_nt", *args)

    # -------------------------------------------------------------- helpers
    def view(self, flat, name):
        o = self.offs[name]
        return flat[o:o + math.prod(self.shapes[name])]

    def pack(self, flat, version=None):
        """Refresh the bf16 weight images from the fp32 master (skipped if `version` unchanged)."""
        if version is not None and version == self._packed_version:
            return
        self._call("es_pack_weights", ptr(flat), ptr(self._pack_tab), self._nmat, _lib.stream())
        self._packed_version = version if version is not None else -1

    def acts(self, n, train):
        key = (n, train)
        if key not in self._acts:
            self._acts[key] = _Acts(self.cfg, n, train, self.device, self.op_dtype)
        return self._acts[key]

    def workspace(self, lane=0):
        """Split-K slabs of the weight-gradient GEMMs (one per backward lane: lanes run concurrently)."""
        if self._ws is None:
            self._ws = {}
        if lane not in self._ws:
            cfg = self.cfg
            D, Hd = cfg.dim, cfg.hidden
            n_tn = max(a * b for a, b in ((3 * D, D), (D, D), (Hd, D), (D, Hd), (D, 3 * cfg.patch * cfg.patch)))
            self._ws[lane] = torch.empty(self.TN_MAX_SPLITS * n_tn + 2 * 1024 * max(Hd, 3 * D), dtype=torch.float32,
                                         device=self.device)
        return self._ws[lane]

    def ln_workspace(self, lane=0):
        """LayerNorm-backward partials (separate from the split-K slabs: the two run on different
        streams when the weight gradients overlap the data-gradient chain)."""
        if self._ws_ln is None:
            self._ws_ln = {}
        if lane not in self._ws_ln:
            self._ws_ln[lane] = torch.empty(2 * LN_BWD_BLOCKS * self.cfg.dim, dtype=torch.float32, device=self.device)
        return self._ws_ln[lane]

    def side_stream(self, tokens=0):
        """The second HIP stream (weak forward beside the train forward; weight gradients beside
        the data-gradient chain): at SIDE_PRIORITY for a step of at least SIDE_PRIORITY_MIN_M train tokens,
        else at the default stream's priority."""
        prio = SIDE_PRIORITY if tokens >= SIDE_PRIORITY_MIN_M else 0
        if self._side is None:
            self._side = {}
        if prio not in self._side:
            self._side[prio] = torch.cuda.Stream(device=self.device, priority=prio)
        return self._side[prio]

    def third_stream(self):
        """A third HIP stream: the small shard's grouped weight gradients beside the two chain lanes."""
        if getattr(self, "_third", None) is None:
            self._third = torch.cuda.Stream(device=self.device)
        return self._third

    # -------------------------------------------------------------- forward
    def forward(self, flat, images_list, train):
        """images_list: fp32 [n_i, 3, S, S] device tensors, processed as one batch (no concat copy).
        Returns fp32 logits [n, C] (head "cls") or the CLS features [n, D] (head "emb"), a view into
        the engine's buffer."""
        cfg = self.cfg
        s = _lib.stream()
        n = sum(int(t.shape[0]) for t in images_list)
        A = self.acts(n, train)
        D, Hd, T, H = cfg.dim, cfg.hidden, cfg.T, cfg.heads
        K0 = 3 * cfg.patch * cfg.patch
        row = 0
        for t in images_list:
            if t.shape[1:] != (3, cfg.img_size, cfg.img_size) or t.dtype not in (torch.float32, torch.uint8):
                raise ValueError(f"expected fp32 (normalised) or uint8 (raw) [n,3,{cfg.img_size},{cfg.img_size}] "
                                 f"images, got {tuple(t.shape)} {t.dtype}")
            t = t.contiguous()
            if t.dtype == torch.uint8:  # ToTensor + Normalize fused into the patch gather
                self._call("es_patch_im2col_u8", ptr(t), *IMAGENET_MEAN, *IMAGENET_STD, ptr(A.patches[row * cfg.np:]),
                     int(t.shape[0]), cfg.img_size, cfg.patch, s)
            else:
                self._call("es_patch_im2col", ptr(t), ptr(A.patches[row * cfg.np:]), int(t.shape[0]), cfg.img_size,
                     cfg.patch, s)
            row += int(t.shape[0])
        x0 = A.x[0]
        pos = self.view(flat, "pos_embed")
        self._call("es_gemm_nt", EPI_PATCH, ptr(A.patches), K0, ptr(self.wb["patch_embed.proj.weight"]), K0,
             ptr(self.view(flat, "patch_embed.proj.bias")), ptr(x0), D, None, ptr(pos), D, n * cfg.np, D, K0,
             cfg.np, s)
        self._call("es_cls_init", ptr(x0), D, ptr(self.view(flat, "cls_token")), ptr(pos), n, T, D, s)
        M = A.M
        prune = self._prune()
        for i in range(cfg.depth):
            b = f"blocks.{i}."
            li = i if train else 0
            xin = A.x[i] if train else A.x[i & 1]
            xout = A.x[i + 1] if train else A.x[(i + 1) & 1]
            xmid, h1, h2 = A.xmid[li], A.h1[li], A.h2[li]
            self._call("es_layernorm_fwd", ptr(xin), D, ptr(self.view(flat, b + "norm1.weight")),
                 ptr(self.view(flat, b + "norm1.bias")), ptr(h1), D, ptr(A.mean1[li]), ptr(A.rstd1[li]), M, D,
                 cfg.eps, s)
            if prune and self.PRUNE_Q and i == cfg.depth - 1:
                # K and V for every token; Q for the CLS rows only, written to their rows of qkv
                wq, bq = self.wb[b + "attn.qkv.weight"], self.view(flat, b + "attn.qkv.bias")
                self._call("es_gemm_nt", EPI_BF16, ptr(h1), D, ptr(wq[D:]), D, ptr(bq[D:]), ptr(A.qkv[li][:, D:]), 3 * D,
                     None, None, 0, M, 2 * D, D, 0, s)
                A.c_h1[:n].copy_(h1[:M].view(n, T, D)[:, 0])
                self._call("es_gemm_nt", EPI_BF16, ptr(A.c_h1), D, ptr(wq[:D]), D, ptr(bq[:D]), ptr(A.qkv[li]), T * 3 * D,
                     None, None, 0, n, D, D, 0, s)
            else:
                self._call("es_gemm_nt", EPI_BF16, ptr(h1), D, ptr(self.wb[b + "attn.qkv.weight"]), D,
                     ptr(self.view(flat, b + "attn.qkv.bias")), ptr(A.qkv[li]), 3 * D, None, None, 0, M, 3 * D, D, 0,
                     s)
            if prune and i == cfg.depth - 1:
                self._last_block_cls_fwd(flat, A, b, li, xin, n, train, s)
                if self.capture is not None:
                    self.capture("fwd_cls", train, i, xin[:M], A.c_xout[:n])
                break
            self._call("es_attn_fwd", ptr(A.qkv[li]), 3 * D, ptr(A.o[li]), D, ptr(A.lse[li]), n, T, H, 64 ** -0.5, s)
            if self.RESID_LN and D == 384 and self.precision == "bf16" and M >= self.RESID_LN_MIN_M:
                self._call("es_gemm_nt_resid_ln", ptr(A.o[li]), D, ptr(self.wb[b + "attn.proj.weight"]), D,
                     ptr(self.view(flat, b + "attn.proj.bias")), ptr(xmid), D, ptr(xin), D,
                     ptr(self.view(flat, b + "norm2.weight")), ptr(self.view(flat, b + "norm2.bias")), ptr(h2), D,
                     ptr(A.mean2[li]), ptr(A.rstd2[li]), M, D, D, cfg.eps, s)
            else:
                self._call("es_gemm_nt", EPI_F32_RESID, ptr(A.o[li]), D, ptr(self.wb[b + "attn.proj.weight"]), D,
                     ptr(self.view(flat, b + "attn.proj.bias")), ptr(xmid), D, None, ptr(xin), D, M, D, D, 0, s)
                self._call("es_layernorm_fwd", ptr(xmid), D, ptr(self.view(flat, b + "norm2.weight")),
                     ptr(self.view(flat, b + "norm2.bias")), ptr(h2), D, ptr(A.mean2[li]), ptr(A.rstd2[li]), M, D,
                     cfg.eps, s)
            if train:
                self._gemm("fc1_fwd", EPI_GELU_D if self.GELU_D else EPI_GELU, ptr(h2), D,
                           ptr(self.wb[b + "mlp.fc1.weight"]), D,
                           ptr(self.view(flat, b + "mlp.fc1.bias")), ptr(A.pre[li]), Hd, ptr(A.act[li]), None, 0, M,
                           Hd, D, 0, s)
            else:
                self._gemm("fc1_fwd_weak", EPI_GELU_ACT, ptr(h2), D, ptr(self.wb[b + "mlp.fc1.weight"]), D,
                           ptr(self.view(flat, b + "mlp.fc1.bias")), ptr(A.act[li]), Hd, None, None, 0, M, Hd, D, 0,
                           s)
            self._call("es_gemm_nt", EPI_F32_RESID, ptr(A.act[li]), Hd, ptr(self.wb[b + "mlp.fc2.weight"]), Hd,
                 ptr(self.view(flat, b + "mlp.fc2.bias")), ptr(xout), D, None, ptr(xmid), D, M, D, Hd, 0, s)
            if self.capture is not None:
                self.capture("fwd", train, i, xin[:M], xout[:M])
        xl = A.x[cfg.depth] if train else A.x[cfg.depth & 1]
        Tl = T  # row stride of the CLS tokens in xl, in tokens
        if prune:
            xl, Tl = A.c_xout, 1
        if cfg.head == "emb":  # CLS features for ModelwEmb's heads (comatch_model.py)
            self._call("es_cls_ln_fwd", ptr(xl), D, Tl, ptr(self.view(flat, "norm.weight")),
                 ptr(self.view(flat, "norm.bias")), ptr(A.fts), D, ptr(A.xhat), ptr(A.rstd_cls), n, D, cfg.eps, s)
            return A.fts
        self._call("es_cls_head_fwd", ptr(xl), D, Tl, ptr(self.view(flat, "norm.weight")), ptr(self.view(flat, "norm.bias")),
             ptr(self.view(flat, "head.weight")), ptr(self.view(flat, "head.bias")), ptr(A.logits),
             cfg.num_classes, ptr(A.xhat), ptr(A.rstd_cls), n, D, cfg.num_classes, cfg.eps, s)
        return A.logits

    def _prune(self):
        """PRUNE_LAST in effect (read at each forward / backward: tests override it per instance);
        the two-lane backward runs every row."""
        return self.PRUNE_LAST

    def _last_block_cls_fwd(self, flat, A, b, li, xin, n, train, s):
        """The last block after its qkv GEMM, on the CLS rows only (PRUNE_LAST): CLS-query attention
        over all keys, then projection (+ the residual read from the CLS rows of xin in place), LN2
        and the MLP on n compact rows -> A.c_xout."""
        cfg = self.cfg
        D, Hd, T, H = cfg.dim, cfg.hidden, cfg.T, cfg.heads
        fv = lambda name: ptr(self.view(flat, name))  # noqa: E731
        self._call("es_attn_cls_fwd", ptr(A.qkv[li]), 3 * D, ptr(A.c_o), D, ptr(A.c_lse), n, T, H, 64 ** -0.5, s)
        self._call("es_gemm_nt", EPI_F32_RESID, ptr(A.c_o), D, ptr(self.wb[b + "attn.proj.weight"]), D,
             fv(b + "attn.proj.bias"), ptr(A.c_xmid), D, None, ptr(xin), T * D, n, D, D, 0, s)
        self._call("es_layernorm_fwd", ptr(A.c_xmid), D, fv(b + "norm2.weight"), fv(b + "norm2.bias"), ptr(A.c_h2), D,
             ptr(A.c_mean2), ptr(A.c_rstd2), n, D, cfg.eps, s)
        if train:
            self._call("es_gemm_nt", EPI_GELU_D if self.GELU_D else EPI_GELU, ptr(A.c_h2), D,
                 ptr(self.wb[b + "mlp.fc1.weight"]), D, fv(b + "mlp.fc1.bias"), ptr(A.c_pre), Hd, ptr(A.c_act), None,
                 0, n, Hd, D, 0, s)
        else:
            self._call("es_gemm_nt", EPI_GELU_ACT, ptr(A.c_h2), D, ptr(self.wb[b + "mlp.fc1.weight"]), D,
                 fv(b + "mlp.fc1.bias"), ptr(A.c_act), Hd, None, None, 0, n, Hd, D, 0, s)
        self._call("es_gemm_nt", EPI_F32_RESID, ptr(A.c_act), Hd, ptr(self.wb[b + "mlp.fc2.weight"]), Hd,
             fv(b + "mlp.fc2.bias"), ptr(A.c_xout), D, None, ptr(A.c_xmid), D, n, D, Hd, 0, s)

    # -------------------------------------------------------------- backward
    def _tn_splits(self, M, N1, N2):
        """0 = the library's automatic split-K sizing for the kernel it picks (es_gemm_tn).  With the
        weight gradients overlapped on the side stream and TN_SHARE < 1, the 384 x 192 tile's launches
        are sized to that share of the CUs (the rest stay free for the data-gradient chain)."""
        if self._tn_shared(M, N1, N2):
            if self._ncu is None:
                self._ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
            tiles = (N1 // 384) * (N2 // 192)
            return max(1, int(self._ncu * self.TN_SHARE) // tiles)
        return 0

    def _tn_shared(self, M, N1, N2):
        """The overlapped weight gradient on the 384 x 192 tile sized to TN_SHARE of the CUs: from the
        F1 batch down to a rank's share at N = 4 (M = 25,216 tokens; the library alone picks that tile
        from M = 65,536).  Same-box A/Bs: N = 2 shard 19.01-19.26 -> 18.15-18.32 ms, N = 4 shard
        10.07-10.09 -> 9.73-9.74 ms (the whole-chip big tile: 18.80-18.96 / 10.25-10.27)."""
        return (self.TN_SHARE < 1.0 and self.overlap and M >= self.TN_SHARE_MIN_M and N1 % 384 == 0
                and N2 % 192 == 0 and self.precision == "bf16")

    def _wgrad(self, dy, N1, x, N2, M, out, bias_out=None, lane=0, ld1=None, ld2=None, label=None):
        """out = dy^T x (weight grad) and, fused, bias_out = column sums of dy (row strides ld1 / ld2,
        default N1 / N2).  `label`: a launch site the bench can time with HIP events (self.probe)."""
        ws = self.workspace(lane)
        splits = self._tn_splits(M, N1, N2)
        need = getattr(_lib.load(), "es_gemm_tn_f32_workspace" if self.precision == "fp32" else "es_gemm_tn_workspace")
        if need(N1, N2, splits) > ws.numel():
            raise RuntimeError(f"wgrad workspace too small for {N1}x{N2} x {splits} splits")
        # the CU-share-sized launches name the 384 x 192 tile explicitly (es_gemm_tn_ex); a process-wide
        # pin (es_set_tn_variant, ENDOSSL_TN_VARIANT) still wins inside the library
        variant = 7 if splits and self._tn_shared(M, N1, N2) else -1
        args = (ptr(dy), ld1 or N1, ptr(x), ld2 or N2, M, N1, N2, splits, ptr(ws), ptr(out), 0, ptr(bias_out))
        self._wgrad_launch(args, variant, M, N1, N2, label)

    def _wgrad_launch(self, args, variant, M, N1, N2, label):
        if self.precision == "fp32":  # parity mode: the fp32 twin (no kernel variants)
            fn, args = "es_gemm_tn", args + (_lib.stream(),)
        else:
            fn, args = "es_gemm_tn_ex", args + (variant, _lib.stream())
        pr = self.probe
        if pr is not None and label is not None and pr["label"] == label:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self._call(fn, *args)
            e1.record()
            pr["events"].append((e0, e1, 2.0 * M * N1 * N2))
        else:
            self._call(fn, *args)

    def _ln_bwd(self, dy, x, mean, rstd, gamma, dres, dx, dxb, dgamma, dbeta, M, lane=0, lddx=None, accumulate=0,
                defer=None):
        """defer (a list): the parameter gradients' partials stay in a workspace of their own, recorded in
        `defer` for one es_ln_param_grads_multi launch later (Engine.DEFER_LN_GRADS)."""
        D = self.cfg.dim
        fn = "es_layernorm_bwd_b16" if dy.dtype == torch.bfloat16 else "es_layernorm_bwd"  # (_f32 in parity mode)
        grid = _lib.load().es_layernorm_bwd_grid(LN_BWD_BLOCKS, M)
        if defer is not None and grid >= 64:  # (one multi-reduce launch takes one column-width class: grid >= 64)
            ws = self.ln_part_workspace(self._lnp_next)  # never reused within a reverse pass (the side stream
            self._lnp_next += 1                           # may reduce a flushed one after the chain moved on)
            self._call(fn, ptr(dy), D, ptr(x), D, ptr(mean), ptr(rstd), ptr(gamma), ptr(dres), D, ptr(dx), lddx or D,
                       ptr(dxb), D, None, None, ptr(ws), LN_BWD_BLOCKS, M, D, 0, _lib.stream())
            defer.append((ws, dgamma, dbeta, grid, accumulate))
            return
        ws = self.ln_workspace(lane)
        self._call(fn, ptr(dy), D, ptr(x), D, ptr(mean), ptr(rstd), ptr(gamma), ptr(dres), D, ptr(dx), lddx or D,
             ptr(dxb), D, ptr(dgamma), ptr(dbeta), ptr(ws), LN_BWD_BLOCKS, M, D, accumulate, _lib.stream())

    def ln_part_workspace(self, k):
        """The k-th deferred LayerNorm backward's partials of a reverse pass (Engine.DEFER_LN_GRADS)."""
        if self._ws_lnp is None:
            self._ws_lnp = []
        while len(self._ws_lnp) <= k:
            self._ws_lnp.append(torch.empty(2 * LN_BWD_BLOCKS * self.cfg.dim, dtype=torch.float32, device=self.device))
        return self._ws_lnp[k]

    def _ln_grads_flush(self, pending):
        """One es_ln_param_grads_multi launch over the deferred LayerNorm backwards in `pending` (then cleared)."""
        if not pending:
            return
        lib = _lib.load()
        esz = lib.es_ln_param_grads_entry_size()
        # es_ln_param_grads_multi takes at most LN_MULTI_MAX entries (the C side's RPM_MAX): larger groups (a
        # bigger GROUP_LAYERS, deeper models) go out as several launches
        for c0 in range(0, len(pending), self.LN_MULTI_MAX):
            chunk = pending[c0:c0 + self.LN_MULTI_MAX]
            raw = (ctypes.c_char * (esz * len(chunk)))()
            for j, (ws, dg, db, grid, acc) in enumerate(chunk):
                ent = (ctypes.c_void_p(ptr(ws)), ctypes.c_void_p(ptr(dg)), ctypes.c_void_p(ptr(db)),
                       ctypes.c_int(grid), ctypes.c_int(self.cfg.dim), ctypes.c_int(acc), ctypes.c_int(0))
                buf = b"".join(bytes(e) for e in ent)
                ctypes.memmove(ctypes.byref(raw, j * esz), buf, len(buf))
            self._call("es_ln_param_grads_multi", ctypes.addressof(raw), len(chunk), _lib.stream())
        pending.clear()

    def backward(self, flat, grad, dlogits=None, dfts=None, zero_grad=True, grad_ready=None):
        """dlogits fp32 [n, C] (head "cls") or dfts fp32 [n, D] (head "emb") for the last train
        forward -> grad (flat fp32).  zero_grad=False when the caller already zeroed `grad` and
        wrote the head gradients into it (the trunk's entries are overwritten either way; the
        final-norm grads are accumulated).  grad_ready(lo, hi, events): called once per block as
        soon as grad[lo:hi] (that block's contiguous parameters) is final -- after the HIP events
        in `events` -- so the caller can start its all-reduce beside the rest of the reverse pass
        (dist.GradBuckets); ranges never handed over are the caller's to finish."""
        cfg = self.cfg
        s = _lib.stream()
        EPI_DH = EPI_BF16 if self.DH_BF16 else EPI_F32  # noqa: N806
        top = dfts if cfg.head == "emb" else dlogits
        if top is None:
            raise ValueError("Engine.backward needs dlogits (cls head) or dfts (emb head)")
        n = int(top.shape[0])
        A = self.acts(n, True)
        if n not in self._grads:
            # two sets: layer i's weight-gradient inputs (dY images) live in set i % 2, so the side
            # stream can still read layer i+1's while the main stream writes layer i's
            self._grads[n] = (_Grads(cfg, n, self.device, self.op_dtype), _Grads(cfg, n, self.device, self.op_dtype))
        G = self._grads[n][0]
        GS = self._grads[n]
        D, Hd, T, H, M = cfg.dim, cfg.hidden, cfg.T, cfg.heads, A.M
        gv = lambda name: self.view(grad, name)  # noqa: E731
        fv = lambda name: self.view(flat, name)  # noqa: E731
        ov = self.overlap
        main = torch.cuda.current_stream(self.device)
        side = self.side_stream(M) if ov else None
        grouped = self._grouped_wgrad(M, grad_ready)
        if grouped:
            # one dY set per layer (+ a spare for layer 0's unused dY of the embedding): the grouped launch
            # at the end reads every layer's weight-gradient inputs
            key = (n, "grouped")
            if key not in self._grads:
                self._grads[key] = [G] + [_Grads(cfg, n, self.device, self.op_dtype) for _ in range(cfg.depth)]
            GS = self._grads[key]
        ovw = ov and not grouped
        nh = n // 2
        lanes = (grouped and ov and self.SHARD_LANES and self.capture is None and n % 2 == 0 and nh > 0
                 and self.precision == "bf16")
        third = self.third_stream() if lanes else None
        problems = []
        layer_wg = self.LAYER_WGRAD and not grouped and self.precision == "bf16" and M >= self.TN_SHARE_MIN_M
        lp = []  # this block's long-axis weight gradients (layer_wg): one grouped launch at the block's end
        # deferred LayerNorm parameter gradients (Engine.DEFER_LN_GRADS): reduced with the weight-gradient launches
        lnd = ([] if self.DEFER_LN_GRADS and grad_ready is None and self.capture is None and not lanes
               and (grouped or layer_wg) else None)
        self._lnp_next = 0

        def wgrad_side(dy, N1, x, N2, Mw, out, bias_out=None, ld1=None, ld2=None, label=None):
            """Weight-gradient GEMM on the side stream once the main stream has produced dY (or, grouped,
            recorded for the one launch after the chain / at the end of the block)."""
            if grouped:
                problems.append((dy, N1, x, N2, Mw, out, bias_out, ld1 or N1, ld2 or N2))
                return
            if (layer_wg and Mw >= self.TN_SHARE_MIN_M and N1 % 384 == 0 and N2 % 192 == 0
                    and (ld1 or N1) % 8 == 0 and (ld2 or N2) % 8 == 0):
                lp.append((dy, N1, x, N2, Mw, out, bias_out, ld1 or N1, ld2 or N2, label))
                return
            if not ov:
                self._wgrad(dy, N1, x, N2, Mw, out, bias_out, ld1=ld1, ld2=ld2, label=label)
                return
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self._wgrad(dy, N1, x, N2, Mw, out, bias_out, ld1=ld1, ld2=ld2, label=label)

        done = {}

        def flush_layer(i):
            """Block i's recorded weight gradients as one grouped split-K launch on the side stream (and the
            LayerNorm parameter gradients deferred so far)."""
            if not lp and not (layer_wg and lnd):
                return
            probs = list(lp)
            lp.clear()

            def run():
                if probs:
                    self._wgrad_layer(probs, i)
                if layer_wg and lnd:
                    self._ln_grads_flush(lnd)
            if ov:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    run()
            else:
                run()

        def block_done(i):
            if self.capture is not None:
                self.capture("bwd", True, i, G.dx[:M])
            if grouped and i > 0 and i % self.GROUP_LAYERS == 0 and problems:
                # these layers' weight gradients as one grouped launch on the side stream (two lanes: a third
                # stream after both), beside the rest of the data-gradient chain (their dY sets are never
                # rewritten within the step)
                if lanes:
                    third.wait_stream(main)
                    third.wait_stream(side)
                    with torch.cuda.stream(third):
                        self._launch_grouped(problems, i)
                elif ov:
                    side.wait_stream(main)
                    with torch.cuda.stream(side):
                        self._launch_grouped(problems, i)
                        if lnd:
                            self._ln_grads_flush(lnd)
                else:
                    self._launch_grouped(problems, i)
                    if lnd:
                        self._ln_grads_flush(lnd)
                problems.clear()
            if grad_ready is None:
                return
            lo = self.offs[f"blocks.{i}.norm1.weight"]
            hi = self.offs[f"blocks.{i + 1}.norm1.weight" if i + 1 < cfg.depth else "norm.weight"]
            evs = [main.record_event()] + ([done[i]] if i in done else [])
            grad_ready(lo, hi, evs)

        # zero_grad: no zero fill of the flat gradient -- every entry of it is written by its first writer of the
        # reverse pass (the head / final-norm kernel with accumulate = 0, the LayerNorm and weight-gradient
        # reductions and the embedding backward overwrite); test_gpu_step.py checks a NaN-filled buffer.  The
        # emb head's final-norm kernel (es_cls_ln_bwd) adds, so that path keeps the fill.
        if zero_grad and cfg.head == "emb":
            grad.zero_()
        prune = self._prune()
        GL = GS[cfg.depth - 1] if grouped else GS[(cfg.depth - 1) % 2]
        # d(loss)/d(CLS tokens after the last block): compact rows (prune) or the CLS rows of G.dx
        dtop, Tt = (GL.c_dx, 1) if prune else (G.dx, T)
        if not prune:
            G.dx.zero_()
        if cfg.head == "emb":
            dfts = dfts.contiguous()
            self._call("es_cls_ln_bwd", ptr(dfts), D, ptr(fv("norm.weight")), ptr(A.xhat), ptr(A.rstd_cls), ptr(dtop), D, Tt,
                 ptr(gv("norm.weight")), ptr(gv("norm.bias")), n, D, s)
        else:
            dlogits = dlogits.contiguous()
            self._call("es_cls_head_bwd_ex", ptr(dlogits), cfg.num_classes, ptr(fv("head.weight")), ptr(fv("norm.weight")),
                 ptr(fv("norm.bias")), ptr(A.xhat), ptr(A.rstd_cls), ptr(G.dyn), ptr(dtop), D, Tt,
                 ptr(gv("head.weight")), ptr(gv("head.bias")), ptr(gv("norm.weight")), ptr(gv("norm.bias")), n, D,
                 cfg.num_classes, 0 if zero_grad else 1, s)
        if self.capture is not None:
            self.capture("dtop", True, cfg.depth - 1, dtop[:n] if prune else G.dx[:M])
        if prune:
            self._call("es_cast_f32_bf16", ptr(GL.c_dx), ptr(GL.c_dxb), n * D, s)
        else:
            self._call("es_cast_f32_bf16", ptr(G.dx), ptr(GL.dxb), M * D, s)
        for i in reversed(range(cfg.depth)):
            b = f"blocks.{i}."
            if grouped:
                Gi, Gn = GS[i], GS[i - 1] if i > 0 else GS[cfg.depth]
            else:
                Gi, Gn = GS[i % 2], GS[(i - 1) % 2]
            if prune and i == cfg.depth - 1:
                # ---- the last block on its CLS rows: MLP, LN2 and projection over n compact rows
                self._call("es_gemm_nt", EPI_MULAUX if self.GELU_D else EPI_DGELU, ptr(Gi.c_dxb), D,
                     ptr(self.wt[b + "mlp.fc2.weight"]), D, None, ptr(Gi.c_dpre), Hd, None, ptr(A.c_pre), Hd, n, Hd,
                     D, 0, s)
                wgrad_side(Gi.c_dxb, D, A.c_act, Hd, n, gv(b + "mlp.fc2.weight"), gv(b + "mlp.fc2.bias"))
                self._call("es_gemm_nt", EPI_DH, ptr(Gi.c_dpre), Hd, ptr(self.wt[b + "mlp.fc1.weight"]), Hd, None,
                     ptr(Gi.c_dh), D, None, None, 0, n, D, Hd, 0, s)
                wgrad_side(Gi.c_dpre, Hd, A.c_h2, D, n, gv(b + "mlp.fc1.weight"), gv(b + "mlp.fc1.bias"))
                # d(xmid) lands on the CLS rows of the full token image dxm_cls (zero elsewhere)
                self._ln_bwd(Gi.c_dh, A.c_xmid, A.c_mean2, A.c_rstd2, fv(b + "norm2.weight"), Gi.c_dx, Gi.dxm_cls,
                             Gi.c_dxmb, gv(b + "norm2.weight"), gv(b + "norm2.bias"), n, lddx=T * D, defer=lnd)
                self._call("es_gemm_nt", EPI_BF16, ptr(Gi.c_dxmb), D, ptr(self.wt[b + "attn.proj.weight"]), D, None,
                     ptr(Gi.c_do), D, None, None, 0, n, D, D, 0, s)
                wgrad_side(Gi.c_dxmb, D, A.c_o, D, n, gv(b + "attn.proj.weight"), gv(b + "attn.proj.bias"))
                self._call("es_attn_cls_bwd", ptr(A.qkv[i]), 3 * D, ptr(A.c_o), D, ptr(A.c_lse), ptr(Gi.c_do), D,
                     ptr(Gi.dqkv), 3 * D, n, T, H, 64 ** -0.5, s)
                self._call("es_gemm_nt", EPI_DH, ptr(Gi.dqkv), 3 * D, ptr(self.wt[b + "attn.qkv.weight"]), 3 * D, None,
                     ptr(G.dh), D, None, None, 0, M, D, 3 * D, 0, s)
                gw, gb = gv(b + "attn.qkv.weight"), gv(b + "attn.qkv.bias")
                if self.PRUNE_Q and n % 32 == 0:
                    # K / V weight gradients over every token; the Q part over the CLS rows, the only
                    # rows with a nonzero dQ (strided views: rows img*T of dqkv and h1)
                    wgrad_side(Gi.dqkv[:, D:], 2 * D, A.h1[i], D, M, gw[D * D:], gb[D:], ld1=3 * D)
                    wgrad_side(Gi.dqkv, D, A.h1[i], D, n, gw[:D * D], gb[:D], ld1=T * 3 * D, ld2=T * D)
                else:
                    wgrad_side(Gi.dqkv, 3 * D, A.h1[i], D, M, gw, gb)
                flush_layer(i)
                if ovw:
                    done[i] = side.record_event()
                self._ln_bwd(G.dh, A.x[i], A.mean1[i], A.rstd1[i], fv(b + "norm1.weight"), Gi.dxm_cls, G.dx, Gn.dxb,
                             gv(b + "norm1.weight"), gv(b + "norm1.bias"), M, defer=lnd)
                block_done(i)
                continue
            if lanes:
                if i == (cfg.depth - 2 if prune else cfg.depth - 1):
                    side.wait_stream(main)  # lane 1 starts from the last block's (or the head's) output gradient
                self._lanes_block(flat, grad, A, G, Gi, Gn, i, n, nh, main, side)
                wgrad_side(Gi.dxb, D, A.act[i], Hd, M, gv(b + "mlp.fc2.weight"), gv(b + "mlp.fc2.bias"))
                wgrad_side(Gi.dpre, Hd, A.h2[i], D, M, gv(b + "mlp.fc1.weight"), gv(b + "mlp.fc1.bias"))
                wgrad_side(Gi.dxmb, D, A.o[i], D, M, gv(b + "attn.proj.weight"), gv(b + "attn.proj.bias"))
                wgrad_side(Gi.dqkv, 3 * D, A.h1[i], D, M, gv(b + "attn.qkv.weight"), gv(b + "attn.qkv.bias"))
                block_done(i)
                continue
            # ---- MLP:  x_{i+1} = xmid + fc2(gelu(fc1(LN2(xmid))))
            cap = self.capture  # test hook: each reverse-pass intermediate as the next op reads it
            if cap is not None:
                cap("b_dxb", True, i, Gi.dxb[:M])
            self._call("es_gemm_nt", EPI_MULAUX if self.GELU_D else EPI_DGELU, ptr(Gi.dxb), D,
                 ptr(self.wt[b + "mlp.fc2.weight"]), D, None, ptr(Gi.dpre), Hd, None, ptr(A.pre[i]), Hd, M, Hd, D, 0, s)
            wgrad_side(Gi.dxb, D, A.act[i], Hd, M, gv(b + "mlp.fc2.weight"), gv(b + "mlp.fc2.bias"))
            self._call("es_gemm_nt", EPI_DH, ptr(Gi.dpre), Hd, ptr(self.wt[b + "mlp.fc1.weight"]), Hd, None, ptr(G.dh),
                 D, None, None, 0, M, D, Hd, 0, s)
            wgrad_side(Gi.dpre, Hd, A.h2[i], D, M, gv(b + "mlp.fc1.weight"), gv(b + "mlp.fc1.bias"), label="fc1_wgrad")
            if cap is not None:
                cap("b_dpre", True, i, Gi.dpre[:M])
                cap("b_dh2", True, i, G.dh[:M])
            self._ln_bwd(G.dh, A.xmid[i], A.mean2[i], A.rstd2[i], fv(b + "norm2.weight"), G.dx, G.dxm, Gi.dxmb,
                         gv(b + "norm2.weight"), gv(b + "norm2.bias"), M, defer=lnd)
            # ---- attention:  xmid = x_i + proj(attn(LN1(x_i)))
            self._call("es_gemm_nt", EPI_BF16, ptr(Gi.dxmb), D, ptr(self.wt[b + "attn.proj.weight"]), D, None, ptr(G.do), D,
                 None, None, 0, M, D, D, 0, s)
            wgrad_side(Gi.dxmb, D, A.o[i], D, M, gv(b + "attn.proj.weight"), gv(b + "attn.proj.bias"))
            if cap is not None:
                cap("b_dxm", True, i, G.dxm[:M], Gi.dxmb[:M])
                cap("b_do", True, i, G.do[:M])
            self._call("es_attn_bwd", ptr(A.qkv[i]), 3 * D, ptr(A.o[i]), D, ptr(A.lse[i]), ptr(G.delta), ptr(G.do), D,
                 ptr(Gi.dqkv), 3 * D, n, T, H, 64 ** -0.5, s)
            self._call("es_gemm_nt", EPI_DH, ptr(Gi.dqkv), 3 * D, ptr(self.wt[b + "attn.qkv.weight"]), 3 * D, None,
                 ptr(G.dh), D, None, None, 0, M, D, 3 * D, 0, s)
            wgrad_side(Gi.dqkv, 3 * D, A.h1[i], D, M, gv(b + "attn.qkv.weight"), gv(b + "attn.qkv.bias"))
            if cap is not None:
                cap("b_dqkv", True, i, Gi.dqkv[:M])
                cap("b_dh1", True, i, G.dh[:M])
            flush_layer(i)
            if ovw:
                done[i] = side.record_event()
                if i + 1 in done:  # set (i-1) % 2 was layer i+1's: its weight gradients must be done
                    main.wait_event(done.pop(i + 1))
            self._ln_bwd(G.dh, A.x[i], A.mean1[i], A.rstd1[i], fv(b + "norm1.weight"), G.dxm, G.dx, Gn.dxb,
                         gv(b + "norm1.weight"), gv(b + "norm1.bias"), M, defer=lnd)
            block_done(i)
        # ---- embedding: x_0 = [cls; patch_embed(img)] + pos
        K0 = 3 * cfg.patch * cfg.patch
        if lanes:
            main.wait_stream(side)  # lane 1's rows of d(loss)/d(x_0)
        self._call("es_embed_bwd", ptr(G.dx), D, ptr(G.dpatch), D, ptr(gv("pos_embed")), ptr(gv("cls_token")), n, T, D, 0,
             s)
        npat = n * cfg.np
        wgrad_side(G.dpatch, D, A.patches, K0, npat, gv("patch_embed.proj.weight"), gv("patch_embed.proj.bias"))
        flush_layer(-1)  # the patch-embedding weight gradient (layer_wg): the backward's last launch
        if grouped:
            self._launch_grouped(problems, 0)
        if lnd:
            self._ln_grads_flush(lnd)
        if ov:
            main.wait_stream(side)
        if lanes:
            main.wait_stream(third)
        return grad

    def _lanes_block(self, flat, grad, A, G, Gi, Gn, i, n, nh, main, side):
        """Block i's data-gradient chain as two lanes (Engine.SHARD_LANES): images [0, nh) on the caller's
        stream, [nh, n) on the side stream, each on its rows of the same buffers (token rows are per image, the
        chain never mixes images).  The LayerNorm parameter gradients are the only sums over both halves: lane 1
        adds its share to lane 0's (accumulate), ordered by an event.  Lane 0 finished block i+1 on main, lane 1
        on side; the embedding backward waits for both."""
        cfg = self.cfg
        D, Hd, T, H = cfg.dim, cfg.hidden, cfg.T, cfg.heads
        EPI_DH = EPI_BF16 if self.DH_BF16 else EPI_F32  # noqa: N806
        b = f"blocks.{i}."
        fv = lambda name: self.view(flat, name)  # noqa: E731
        gv = lambda name: self.view(grad, name)  # noqa: E731
        ev = {}
        for ln, st in ((0, main), (1, side)):
            i0, nl = (0, nh) if ln == 0 else (nh, n - nh)
            r0, Ml = i0 * T, nl * T
            with torch.cuda.stream(st):
                s = _lib.stream()
                rp = lambda t, r0=r0: ptr(t[r0:])  # noqa: E731
                self._call("es_gemm_nt", EPI_MULAUX if self.GELU_D else EPI_DGELU, rp(Gi.dxb), D,
                           ptr(self.wt[b + "mlp.fc2.weight"]), D, None, rp(Gi.dpre), Hd, None, rp(A.pre[i]), Hd, Ml, Hd,
                           D, 0, s)
                self._call("es_gemm_nt", EPI_DH, rp(Gi.dpre), Hd, ptr(self.wt[b + "mlp.fc1.weight"]), Hd, None,
                           rp(G.dh), D, None, None, 0, Ml, D, Hd, 0, s)
                if ln == 1:
                    st.wait_event(ev["ln2"])
                self._ln_bwd(G.dh[r0:], A.xmid[i][r0:], A.mean2[i][r0:], A.rstd2[i][r0:], fv(b + "norm2.weight"),
                             G.dx[r0:], G.dxm[r0:], Gi.dxmb[r0:], gv(b + "norm2.weight"), gv(b + "norm2.bias"), Ml,
                             lane=ln, accumulate=ln)
                if ln == 0:
                    ev["ln2"] = st.record_event()
                self._call("es_gemm_nt", EPI_BF16, rp(Gi.dxmb), D, ptr(self.wt[b + "attn.proj.weight"]), D, None,
                           rp(G.do), D, None, None, 0, Ml, D, D, 0, s)
                self._call("es_attn_bwd", rp(A.qkv[i]), 3 * D, rp(A.o[i]), D, ptr(A.lse[i][i0 * H * T:]),
                           ptr(G.delta[i0 * H * T:]), rp(G.do), D, rp(Gi.dqkv), 3 * D, nl, T, H, 64 ** -0.5, s)
                self._call("es_gemm_nt", EPI_DH, rp(Gi.dqkv), 3 * D, ptr(self.wt[b + "attn.qkv.weight"]), 3 * D, None,
                           rp(G.dh), D, None, None, 0, Ml, D, 3 * D, 0, s)
                if ln == 1:
                    st.wait_event(ev["ln1"])
                self._ln_bwd(G.dh[r0:], A.x[i][r0:], A.mean1[i][r0:], A.rstd1[i][r0:], fv(b + "norm1.weight"),
                             G.dxm[r0:], G.dx[r0:], Gn.dxb[r0:], gv(b + "norm1.weight"), gv(b + "norm1.bias"), Ml,
                             lane=ln, accumulate=ln)
                if ln == 0:
                    ev["ln1"] = st.record_event()

    def _wgrad_layer(self, problems, layer):
        """One es_gemm_tn_big_grouped launch (+ its reduce) over a block's weight gradients, on the
        current stream.  Sized to LAYER_TN_SHARE of the CUs while the data-gradient chain still runs
        beside it; the first block's (the last launch of the backward: nothing left beside it) and the
        serial engine's to the whole chip.  The problem table travels in the kernel arguments (no
        host->device copy; capturable)."""
        lib = _lib.load()
        if self._ncu is None:
            self._ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        share = self.LAYER_TN_SHARE if (self.overlap and layer > 0) else 1.0  # block 0 / the embedding: chip
        target = max(1, int(self._ncu * share))
        n = len(problems)
        tab = (_TNProblem * n)()
        for e, (dy, N1, x, N2, Mw, out, bias, ld1, ld2, _) in zip(tab, problems):
            e.dy, e.x, e.out, e.bias_out = ptr(dy), ptr(x), ptr(out), ptr(bias) if bias is not None else None
            e.M, e.N1, e.N2, e.ld1, e.ld2 = Mw, N1, N2, ld1, ld2
        ws = self.workspace(0)
        need = lib.es_gemm_tn_big_grouped_workspace(ctypes.byref(tab), n, target)
        if need > ws.numel():
            raise RuntimeError(f"grouped weight-gradient workspace too small: {need} > {ws.numel()} floats")
        raw = ctypes.create_string_buffer(lib.es_gemm_tn_big_grouped_table_bytes(n))
        dims = (ctypes.c_int * 3)()
        rc = lib.es_gemm_tn_big_grouped_prepare(ctypes.byref(tab), n, target, ptr(ws), ws.numel(), raw, dims)
        if rc != 0:
            raise _lib.EndosslLibraryError(f"es_gemm_tn_big_grouped_prepare: status {rc}")
        pr = self.probe
        # probed at the launches sized like the timed ones: the CU-share-sized blocks (or every block of the
        # serial engine), not the first block's whole-chip launch at the end of an overlapped backward
        if pr is not None and any(q[9] == pr["label"] for q in problems) and (layer > 0 or not self.overlap):
            flop = sum(2.0 * q[4] * q[1] * q[3] for q in problems)
            # timed by the kernels' own start / end (hipExtLaunchKernelGGL events), as a kernel trace sees them
            e0, e1 = _lib.KernelEvent(), _lib.KernelEvent()
            call("es_gemm_tn_big_grouped_timed", raw, n, dims, e0.handle, e1.handle, _lib.stream())
            pr["events"].append((e0, e1, flop))
            pr["layer_kernel"] = (f"es_gemm_tn_big_grouped: one block's {n} weight-gradient GEMMs "
                                  f"({'+'.join(str(q[1]) + 'x' + str(q[3]) for q in problems)}) over M={problems[0][4]} "
                                  f"tokens, {dims[0]} workgroups of 384x192, then one reduce launch")
            pr["layer_bytes"] = sum(2.0 * q[4] * (q[1] + q[3]) + 4.0 * q[1] * q[3] + (4.0 * q[1] if q[6] is not None else 0)
                                    for q in problems)
        else:
            call("es_gemm_tn_big_grouped", raw, n, dims, _lib.stream())

    def _grouped_wgrad(self, M, grad_ready):
        if self.precision != "bf16" or grad_ready is not None:  # per-block hand-over needs per-layer launches
            return False
        return self.GROUP_WGRAD == "1" or (self.GROUP_WGRAD == "auto" and M < self.GROUP_WGRAD_MAX_M)

    def _launch_grouped(self, problems, slot):
        """One es_gemm_tn_grouped launch over the recorded weight-gradient GEMMs (longest token axis
        first).  The table's pointers are stable for a batch size (cached buffers), so the device copy
        (one per launch slot of the step) is re-made only when its bytes change."""
        problems = sorted(problems, key=lambda q: -q[4])
        tab = (_TNProblem * len(problems))()
        for e, (dy, N1, x, N2, Mw, out, bias, ld1, ld2) in zip(tab, problems):
            e.dy, e.x, e.out, e.bias_out = ptr(dy), ptr(x), ptr(out), ptr(bias) if bias is not None else None
            e.M, e.N1, e.N2, e.ld1, e.ld2 = Mw, N1, N2, ld1, ld2
        lib = _lib.load()
        tiles = lib.es_gemm_tn_grouped_prepare(ctypes.byref(tab), len(problems))
        if tiles <= 0:
            raise _lib.EndosslLibraryError(f"es_gemm_tn_grouped_prepare: status {tiles}")
        raw = bytes(tab)
        if not hasattr(self, "_gtab"):
            self._gtab = {}
        cache = self._gtab.get(slot)
        if cache is None or cache[0] != raw:
            if torch.cuda.is_current_stream_capturing():
                # a blocking host->device copy cannot be captured: the eager step that precedes every
                # capture (FixMatch._run_graph) uploads the identical table, so a miss here means the
                # buffers moved between that step and the capture
                raise RuntimeError("grouped weight-gradient table changed during hipGraph capture; run one eager "
                                   "step of this shape first")
            dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device, non_blocking=False)
            self._gtab[slot] = cache = (raw, dev)
        pr = self.probe
        flop = sum(2.0 * q[4] * q[1] * q[3] for q in problems)
        if pr is not None and pr["label"] == "fc1_wgrad":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call("es_gemm_tn_grouped", ptr(cache[1]), len(problems), tiles, _lib.stream())
            e1.record()
            pr["events"].append((e0, e1, flop))
            pr["kernel"] = f"es_gemm_tn_grouped ({len(problems)} weight-gradient GEMMs, {tiles} tiles)"
        else:
            call("es_gemm_tn_grouped", ptr(cache[1]), len(problems), tiles, _lib.stream())


    def head_backward(self, flat, grad, dlogits, train=False):
        """IS_FREEZE (code/fixmatch.py:40-48: every parameter frozen but `model.fc`, timm's `head`):
        grad <- d(loss)/d(head.weight, head.bias) only, from the CLS features the forward (train or
        inference form) normalised; every other entry of grad is zero, so the fused Adam sweep leaves
        the frozen parameters exactly unchanged (zero gradient, zero moments)."""
        cfg = self.cfg
        if cfg.head != "cls":
            raise ValueError("head_backward is the classifier-head model's; the emb-head model runs its heads' "
                             "backward in comatch_model.EmbHeads")
        n, D, C = int(dlogits.shape[0]), cfg.dim, cfg.num_classes
        A = self.acts(n, train)
        if getattr(self, "_hb", None) is None or self._hb[0].shape[0] < n:
            z = lambda *sh: torch.zeros(*sh, dtype=torch.float32, device=self.device)  # noqa: E731
            self._hb = (z(n, D), z(n, D), z(D), z(D))  # dyn, dx (CLS rows), frozen-norm gradients
        dyn, dx, gnw, gnb = self._hb
        grad.zero_()
        self._call("es_cls_head_bwd", ptr(dlogits.contiguous()), C, ptr(self.view(flat, "head.weight")),
                   ptr(self.view(flat, "norm.weight")), ptr(self.view(flat, "norm.bias")), ptr(A.xhat),
                   ptr(A.rstd_cls), ptr(dyn), ptr(dx), D, 1, ptr(self.view(grad, "head.weight")),
                   ptr(self.view(grad, "head.bias")), ptr(gnw), ptr(gnb), n, D, C, _lib.stream())
        return grad


class _ViTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, module, *params):
        ctx.module = module
        ctx.n = int(x.shape[0])
        logits = module.engine().forward(module.flat, [x], train=True)
        return logits.clone()

    @staticmethod
    def backward(ctx, dlogits):
        m = ctx.module
        g = m.engine().backward(m.flat, m.flat_grad, dlogits.float())
        return (None, None) + tuple(m.engine().view(g, name).view(shape) for name, shape in m.layout)


class NativeViT(nn.Module):
    """timm-compatible VisionTransformer whose compute runs in libendossl_hip.so."""

    def __init__(self, cfg=None, seed=None, **kw):
        super().__init__()
        self.cfg = cfg if cfg is not None else ViTConfig(**kw)
        self.layout, self.offs, self.numel = param_layout(self.cfg)
        flat = torch.zeros(self.numel, dtype=torch.float32)
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        timm_init_(flat, self.cfg, self.layout, self.offs, generator=gen)
        self._set_flat(flat)
        self._engine = None
        self.precision = "bf16"  # "fp32": parity mode (Engine.PARITY_NAMES)
        self.version = 0  # bumped whenever the fp32 master changes (bf16 images re-packed lazily)

    # parameters are views into one flat buffer --------------------------------------------
    def _set_flat(self, flat):
        self.flat = flat
        self.flat_grad = torch.zeros_like(flat)
        for name, shape in self.layout:
            view = flat[self.offs[name]:self.offs[name] + math.prod(shape)].view(shape)
            mod, attr = self._resolve(name)
            p = nn.Parameter(view, requires_grad=True)
            mod._parameters[attr] = p

    def _resolve(self, name):
        parts = name.split(".")
        mod = self
        for p in parts[:-1]:
            if p not in mod._modules:
                mod._modules[p] = nn.Module()
            mod = mod._modules[p]
        return mod, parts[-1]

    def _apply(self, fn, recurse=True):
        new = fn(self.flat)
        if new is not self.flat:
            self._set_flat(new.contiguous())
            self._engine = None
        return self

    def __deepcopy__(self, memo):
        other = NativeViT.__new__(NativeViT)
        nn.Module.__init__(other)
        other.cfg, other.layout, other.offs, other.numel = self.cfg, self.layout, self.offs, self.numel
        other._set_flat(self.flat.detach().clone())
        other._engine = None
        other.precision = self.precision
        other.version = 0
        other.train(self.training)
        return other

    def set_precision(self, precision):
        """"bf16" (production: bf16 MFMA operands, fp32 accumulation / master weights) or "fp32"
        (parity mode: every operand fp32, csrc/parity.hip)."""
        if precision not in ("bf16", "fp32"):
            raise ValueError(precision)
        if precision != self.precision:
            self.precision, self._engine = precision, None
        return self

    def engine(self):
        if self._engine is None or self._engine.device != self.flat.device:
            if not self.flat.is_cuda:
                raise _lib.EndosslCallError("NativeViT runs on the MI355X only: move it to a cuda device first")
            self._engine = Engine(self.cfg, self.flat.device, precision=getattr(self, "precision", "bf16"))
        return self._engine

    @property
    def fc(self):  # code/fixmatch.py:48 freezes `model.fc`; timm ViTs call it `head`
        return self.head

    def no_weight_decay(self):
        """timm 0.5.4 VisionTransformer.no_weight_decay (the second Adam param group's names,
        code/optimizer.py:38-41)."""
        return {"pos_embed", "cls_token", "dist_token"}

    def mark_updated(self):
        self.version += 1

    def load_state_dict(self, state_dict, strict=True):
        r = super().load_state_dict(state_dict, strict=strict)
        self.mark_updated()
        return r

    def forward(self, x):
        eng = self.engine()
        eng.pack(self.flat, self.version)
        if torch.is_grad_enabled() and self.training and any(p.requires_grad for p in self.parameters()):
            params = [self.get_parameter(name) for name, _ in self.layout]
            return _ViTFunction.apply(x, self, *params)
        return eng.forward(self.flat, [x], train=False).clone()
