"""Native Conformer -- SemiFormer's backbone on MI355X kernels.

Reference: `Conformer` (code/models/conformer.py:359-445) with ConvBlock (:75-144), FCUDown
(:147-170), FCUUp (:173-194), ConvTransBlock (:250-356) and the ViT Block (:55-72); built by
code/build.py:135-142 as Conformer-Ti (patch 16, channel_ratio 1, embed 384, depth 12, 6 heads,
qkv_bias).  `model(x) -> (conv_logits, trans_logits)` as SemiFormer expects (code/semiformer.py:122).

MI355X-first layout:
  * parameters live in ONE fp32 flat buffer in the reference's state_dict order (checkpoints
    interchange; the fused Adam + EMA sweep of optim.hip updates all of them in one pass); the
    BatchNorm running statistics are ordinary buffers of the BN submodules;
  * the CNN branch keeps NHWC maps and runs on conv.hip (BatchNorm2d with fused residual +
    ReLU, pools, nearest upsampling, fp32 implicit-GEMM convolutions) and conv_bf16.hip (the convs
    whose channel counts are multiples of 32, on bf16 operands: every conv of Conformer-B but the
    3-channel stem; set_conv_precision("fp32") is the parity mode).  When every conv after the stem
    takes the bf16 kernels (Conformer-B: map_bf16) the activation AND gradient maps after the stem's
    max-pool are bf16 -- this repo's own bf16-storage contract: the reference runs its conv / BatchNorm
    chain in fp32 (no autocast); parity for it is per conv against the bf16-rounded-operand contract
    (tests/test_gpu_convs.py) and ENDOSSL_MAP_BF16=0 keeps fp32 maps --, BatchNorm statistics and every
    reduction in fp32; otherwise fp32 maps; the transformer branch is a
    [tokens, D] fp32 residual stream padded to 256 rows (zero pad) and runs on the same bf16 MFMA
    kernels as the ViT (gemm / attention / layernorm); the FCU bridges read and write token rows
    in place through element strides (no transposes);
  * every op is a torch.autograd.Function over the C-ABI; the backward writes parameter gradients
    straight into the flat gradient buffer (each parameter is used once per forward, so every
    launch overwrites its slice), which the native Adam reads.  PyTorch provides the autograd
    graph, device memory and streams only.
"""
import ctypes
import math
import os
from copy import deepcopy

import torch
import torch.nn as nn

from . import _lib, dist
from ._lib import call, ptr
from .vit import IMAGENET_MEAN, IMAGENET_STD

EPI_BF16, EPI_GELU, EPI_F32_RESID, EPI_DGELU, EPI_F32 = 0, 1, 2, 3, 4
EPI_GELU_ACT, EPI_GELU_D, EPI_MULAUX = 6, 7, 8
BN_EPS_BLOCK, BN_EPS_STEM, LN_EPS, LN_EPS_TRANS_NORM = 1e-6, 1e-5, 1e-6, 1e-5
BN_MOMENTUM = 0.1


def _rup(x, m):
    return (x + m - 1) // m * m


class ConformerConfig:
    def __init__(self, img_size=224, patch=16, base_channel=64, channel_ratio=1, embed_dim=384, depth=12, heads=6,
                 mlp_ratio=4.0, num_classes=23, num_med_block=0):
        if depth % 3:
            raise ValueError("Conformer depth must be a multiple of 3 (code/models/conformer.py:366)")
        if num_med_block:
            raise NotImplementedError("num_med_block > 0 (Med_ConvBlock) is not used by build.py's Conformer")
        if embed_dim != heads * 64 or embed_dim % 128:
            raise ValueError("the transformer kernels assume head_dim 64 and embed_dim % 128 == 0")
        self.img_size, self.patch, self.base, self.ratio = img_size, patch, base_channel, channel_ratio
        self.dim, self.depth, self.heads, self.num_classes = embed_dim, depth, heads, num_classes
        self.hidden = int(embed_dim * mlp_ratio)
        self.stem = img_size // 4                 # after conv1 (s2) and the max-pool (s2)
        self.dw = patch // 4
        self.grid = self.stem // self.dw
        self.np = self.grid * self.grid
        self.T = self.np + 1
        s1 = base_channel * channel_ratio
        self.s1, self.s3 = s1, 4 * s1

    def stages(self):
        """(name, inplanes, outplanes, res_conv, stride, dw_stride, last_fusion), code/models/conformer.py:385-416."""
        s1, dw = self.s1, self.dw
        out, fin = [], self.depth // 3 + 1
        for i in range(2, fin):
            out.append((f"conv_trans_{i}", s1, s1, False, 1, dw, False))
        s2 = 2 * s1
        init, fin = fin, fin + self.depth // 3
        for i in range(init, fin):
            out.append((f"conv_trans_{i}", s1 if i == init else s2, s2, i == init, 2 if i == init else 1, dw // 2,
                        False))
        s3 = 2 * s2
        init, fin = fin, fin + self.depth // 3
        for i in range(init, fin):
            out.append((f"conv_trans_{i}", s2 if i == init else s3, s3, i == init, 2 if i == init else 1, dw // 4,
                        i == self.depth))
        return out


# ------------------------------------------------------------------------------------ layout
def _bn_entries(pre, C):
    return [(pre + "weight", (C,), "p"), (pre + "bias", (C,), "p"), (pre + "running_mean", (C,), "rm"),
            (pre + "running_var", (C,), "rv"), (pre + "num_batches_tracked", (), "nbt")]


def _conv_block_entries(pre, inp, outp, res_conv):
    med = outp // 4
    out = [(pre + "conv1.weight", (med, inp, 1, 1), "p")] + _bn_entries(pre + "bn1.", med)
    out += [(pre + "conv2.weight", (med, med, 3, 3), "p")] + _bn_entries(pre + "bn2.", med)
    out += [(pre + "conv3.weight", (outp, med, 1, 1), "p")] + _bn_entries(pre + "bn3.", outp)
    if res_conv:
        out += [(pre + "residual_conv.weight", (outp, inp, 1, 1), "p")] + _bn_entries(pre + "residual_bn.", outp)
    return out


def _block_entries(pre, D, Hd):
    return [(pre + "norm1.weight", (D,), "p"), (pre + "norm1.bias", (D,), "p"),
            (pre + "attn.qkv.weight", (3 * D, D), "p"), (pre + "attn.qkv.bias", (3 * D,), "p"),
            (pre + "attn.proj.weight", (D, D), "p"), (pre + "attn.proj.bias", (D,), "p"),
            (pre + "norm2.weight", (D,), "p"), (pre + "norm2.bias", (D,), "p"),
            (pre + "mlp.fc1.weight", (Hd, D), "p"), (pre + "mlp.fc1.bias", (Hd,), "p"),
            (pre + "mlp.fc2.weight", (D, Hd), "p"), (pre + "mlp.fc2.bias", (D,), "p")]


def conformer_layout(cfg):
    """(name, shape, kind) in the reference Conformer's state_dict order (module registration order
    of code/models/conformer.py:362-411); kind p = parameter, rm / rv / nbt = BatchNorm buffers."""
    D, C = cfg.dim, cfg.num_classes
    out = [("cls_token", (1, 1, D), "p"), ("trans_norm.weight", (D,), "p"), ("trans_norm.bias", (D,), "p"),
           ("trans_cls_head.weight", (C, D), "p"), ("trans_cls_head.bias", (C,), "p"),
           ("conv_cls_head.weight", (C, cfg.s3), "p"), ("conv_cls_head.bias", (C,), "p"),
           ("conv1.weight", (64, 3, 7, 7), "p")] + _bn_entries("bn1.", 64)
    out += _conv_block_entries("conv_1.", 64, cfg.s1, True)
    out += [("trans_patch_conv.weight", (D, 64, cfg.dw, cfg.dw), "p"), ("trans_patch_conv.bias", (D,), "p")]
    out += _block_entries("trans_1.", D, cfg.hidden)
    for name, inp, outp, res_conv, _, _, last in cfg.stages():
        pre = name + "."
        med = outp // 4
        out += _conv_block_entries(pre + "cnn_block.", inp, outp, res_conv)
        out += _conv_block_entries(pre + "fusion_block.", outp, outp, last)
        out += [(pre + "squeeze_block.conv_project.weight", (D, med, 1, 1), "p"),
                (pre + "squeeze_block.conv_project.bias", (D,), "p"),
                (pre + "squeeze_block.ln.weight", (D,), "p"), (pre + "squeeze_block.ln.bias", (D,), "p"),
                (pre + "expand_block.conv_project.weight", (med, D, 1, 1), "p"),
                (pre + "expand_block.conv_project.bias", (med,), "p")]
        out += _bn_entries(pre + "expand_block.bn.", med)
        out += _block_entries(pre + "trans_block.", D, cfg.hidden)
    return out


def init_conformer_(flat, layout, offs, generator=None):
    """Conformer._init_weights (code/models/conformer.py:396-411): Linear trunc_normal(.02) / zero
    bias, LayerNorm and BatchNorm 1 / 0, Conv2d kaiming_normal(fan_out, relu), conv biases keep the
    PyTorch default U(+-1/sqrt(fan_in)), cls_token trunc_normal(.02)."""
    with torch.no_grad():
        for name, shape, kind in layout:
            if kind != "p":
                continue
            t = flat[offs[name]:offs[name] + math.prod(shape)].view(shape)
            if name == "cls_token" or (len(shape) == 2):
                nn.init.trunc_normal_(t, std=0.02, generator=generator)
            elif len(shape) == 4:
                nn.init.kaiming_normal_(t, mode="fan_out", nonlinearity="relu", generator=generator)
            elif name.endswith("weight"):
                t.fill_(1.0)
            else:
                wname = name[:-len("bias")] + "weight"
                wshape = [s for n, s, _ in layout if n == wname][0]
                if len(wshape) == 4:  # Conv2d bias: PyTorch default
                    bound = 1.0 / math.sqrt(math.prod(wshape[1:]))
                    nn.init.uniform_(t, -bound, bound, generator=generator)
                else:
                    t.zero_()


# ------------------------------------------------------------------------------------ ops
def _s():
    return _lib.stream()


# Conv weight / bias gradients on a side HIP stream beside the data-gradient chain (the S1 backward
# is otherwise one serial stream of mostly small, latency-bound launches).  Their inputs are
# record_stream'ed so the caching allocator keeps them until the side stream is done.  The first
# such launch of a backward pass queues an autograd final callback that makes the backward's stream
# wait for the side stream, so whatever runs after `backward()` returns (the all-reduce, the
# optimizer, a test reading .grad) sees complete gradients.
CONV_DW_SIDE = True
_wgrad_streams = {}
_join_queued = set()


def _queue_join(main, side):
    key = (main.device, main.cuda_stream)
    if key in _join_queued:
        return
    _join_queued.add(key)

    def _join():
        main.wait_stream(side)
        _join_queued.discard(key)
    torch.autograd.Variable._execution_engine.queue_callback(_join)


# The CNN branch and the transformer branch of each ConvTransBlock run on two HIP streams (forward;
# autograd then runs each node's backward on its forward stream, so the backward overlaps too):
# after the cnn_block's conv2 / bn2 produce x2, FCUDown -> transformer block -> FCUUp run on the
# branch stream while the cnn_block's conv3 / residual / bn3 tail runs on the caller's stream; the
# fusion block joins them (code/models/conformer.py:334-357 data flow, unchanged arithmetic).
BRANCH_STREAMS = True
_branch_streams = {}
# every conv weight's bf16 images packed in ONE launch per parameter version (NativeConformer.conv_pack) instead
# of one launch per weight at its first use: 96 launches fewer per S1 step; same box, interleaved (r05,
# scripts/gpu_r5k.sh): S1 139.16 / 139.89 / 139.30 vs 139.43 / 139.52 / 139.12 ms, P0 within its noise -- kept for
# the launch count (the small-batch P0 / shard steps are launch-bound), not for a measured gain
CONV_PACK_MULTI = True
# HIP priorities of the branch stream and the weight-gradient stream (0 = the default stream's, -1 = higher).
# S1 same box (profiles/r04_stream_priority.txt): both 0 139.81 / 140.01 ms, branch -1
# 139.53 / 139.00, weight gradients -1 140.26 / 139.92, both -1 139.21 / 139.20
BRANCH_PRIORITY = -1
WGRAD_PRIORITY = 0


def _branch_stream(device):
    st = _branch_streams.get(device)
    if st is None:
        st = _branch_streams[device] = torch.cuda.Stream(device=device, priority=BRANCH_PRIORITY)
    return st


def _own(t):
    """Mark a tensor handed across streams (an autograd gradient, a branch output) as used by the
    current stream, so the caching allocator does not recycle it before this stream's kernels ran."""
    if t is not None and t.is_cuda:
        t.record_stream(torch.cuda.current_stream(t.device))


def _wgrad_stream(device):
    st = _wgrad_streams.get(device)
    if st is None:
        st = _wgrad_streams[device] = torch.cuda.Stream(device=device, priority=WGRAD_PRIORITY)
    return st


def join_wgrad_stream(device=None):
    """Make the current stream wait for the side-stream weight gradients (no-op if none ran)."""
    if not torch.cuda.is_available():
        return
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    st = _wgrad_streams.get(dev)
    if st is not None:
        torch.cuda.current_stream(dev).wait_stream(st)


def _zero_pad(t, rows):
    """Zero rows [rows, len) of a token-row buffer (the GEMM pad rows) and return it."""
    if t.shape[0] > rows:
        t[rows:].zero_()
    return t


class _Map:
    """An NHWC view: tensor t, element offset, (N, H, W, C) and element strides (n, h, w, c)."""

    def __init__(self, t, N, H, W, C, sn=None, sh=None, sw=None, sc=1, off=0):
        self.t, self.N, self.H, self.W, self.C = t, N, H, W, C
        self.sn = sn if sn is not None else H * W * C
        self.sh = sh if sh is not None else W * C
        self.sw = sw if sw is not None else C
        self.sc, self.off = sc, off

    def p(self):
        return ptr(self.t) + self.t.element_size() * self.off

    @staticmethod
    def nhwc(t):
        N, H, W, C = t.shape
        return _Map(t, N, H, W, C)


# share of the CUs the transformer blocks' overlapped weight gradients are sized to (Engine.TN_SHARE's
# counterpart; 1 = the library's whole-chip sizing): S1 195.46 / 195.46 -> 193.26 / 193.38 ms same-box A/B)
CONF_TN_SHARE = 0.5


# a transformer block's four weight gradients (fc2, fc1, proj, qkv) as ONE es_gemm_tn_big_grouped launch (384 x 192
# tiles, split-K over the tokens) plus one reduce, issued on the side stream once the block's last data gradient
# is made -- instead of four es_gemm_tn launches on the 128 x 128 tile (Conformer-B / 384: 938 us of weight
# gradients per block alone on the chip); sized to CONF_TN_SHARE of the CUs beside the branch streams.  Off: S1
# wall neutral (126.5 vs 126.6 ms, the side stream already hid the per-Linear launches), and at one split per tile
# (96 tiles on a 128-workgroup share) its fp32 chains over 36,928 tokens put the proj / qkv weight gradients at
# 1.05-1.16e-5 of the exact product of the device's own inputs, above tests/test_gpu_s1_blocks.py's 1e-5 bar
CONF_TN_GROUPED = False


def _wgrad_grouped(m, probs, M, target, k):
    """One es_gemm_tn_big_grouped launch (+ its reduce) on the current stream over probs = [(dy, N1, x, N2,
    weight name, bias name)]: out / bias gradients overwritten (as es_gemm_tn with accumulate 0)."""
    from .vit import _TNProblem
    lib = _lib.load()
    n = len(probs)
    tab = (_TNProblem * n)()
    for e, (dy, N1, x, N2, wname, bname) in zip(tab, probs):
        e.dy, e.x, e.out = ptr(dy), ptr(x), ptr(m.gview(wname))
        e.bias_out = ptr(m.gview(bname)) if bname else None
        e.M, e.N1, e.N2, e.ld1, e.ld2 = M, N1, N2, N1, N2
    need = lib.es_gemm_tn_big_grouped_workspace(ctypes.byref(tab), n, target)
    ws = m.bwd_scratch(f"tn_grouped_ws/{k}", (max(int(need), 1),), torch.float32)
    raw = ctypes.create_string_buffer(lib.es_gemm_tn_big_grouped_table_bytes(n))
    dims = (ctypes.c_int * 3)()
    rc = lib.es_gemm_tn_big_grouped_prepare(ctypes.byref(tab), n, target, ptr(ws), ws.numel(), raw, dims)
    if rc != 0:
        raise _lib.EndosslLibraryError(f"es_gemm_tn_big_grouped_prepare: status {rc}")
    call("es_gemm_tn_big_grouped", raw, n, dims, _s())


def _tn_splits(M, N1, N2):
    """0: es_gemm_tn sizes the split-K for the kernel it picks (as the ViT engine, Engine._tn_splits)."""
    return 0


# CNN-branch conv operands in bf16 (csrc/conv_bf16.hip: v_mfma_f32_16x16x32_bf16, fp32 maps and
# accumulation) wherever both channel counts are multiples of 32; ENDOSSL_CONV_BF16=0 (or
# NativeConformer.set_conv_precision("fp32")) keeps every conv on conv.hip's fp32 MFMA kernels.
CONV_BF16 = os.environ.get("ENDOSSL_CONV_BF16", "1") != "0"
# train-mode BatchNorm statistics of a bf16 conv's output computed in the conv's epilogue
# (es_conv2d_fwd_bf16_bnstats -> es_bn2d_fwd_partials): no two statistics passes over the map
BN_STATS_FUSED = True
# the backward of a train-mode ReLU BatchNorm without residual rebuilds its mask from x instead of reading y
BN_Y_FREE = True
# a ConvBlock input's two gradient contributions (conv1, residual) summed in place (_GradSink)
GRAD_SINKS = True
# ... and the token buffer's two consumers (a block's FCUUp conv, the next block's FCUDown), _trans_branch
TOKEN_SINK = True
# a train-mode BatchNorm + ReLU whose output feeds ONE bf16 conv (a ConvBlock's bn1 -> conv2 without the FCUUp
# add, and bn2 -> conv3 where x2 has no other consumer) is applied by that conv's gathers instead of being
# written as a map (_BNConvFn); False materialises it (bn, then conv)
BN_CONV_FUSED = True
# ... for k x k convs too (bn1 -> conv2, 3 x 3): off.  Each input pixel is gathered k^2 times and the BatchNorm
# parameters cost the gather kernels a wave per SIMD: at the Conformer-B/384 shapes (scripts/convb_bench.py --bnin)
# the 3 x 3 forward takes 342 / 210 / 219 us fused vs 246 / 167 / 171 plain (stages 1-3) and its weight gradient
# 632 / 515 / 570 vs 522 / 302 / 363, more than the BatchNorm apply it saves; the 1 x 1 convs lose 4-18 % (fwd) and
# 4-27 % (weight gradient).  S1, same box, interleaved (scripts/gpu_r5o.sh): every pair fused 138.56 / 138.86 /
# 138.76 ms, 1 x 1 only 138.46 / 138.12 / 137.80, none 138.33 / 138.27 / 138.69
BN_CONV_FUSED_KXK = False
# bf16 activation / gradient maps in the CNN branch when every conv after the stem runs on conv_bf16.hip
# (NativeConformer.map_bf16); ENDOSSL_MAP_BF16=0 keeps fp32 maps with bf16 conv operands
MAP_BF16 = os.environ.get("ENDOSSL_MAP_BF16", "1") != "0"


def _fl(t):
    """1 for a bf16 map, 0 for fp32 (the _ex entry points' flag bit)."""
    return 1 if t.dtype == torch.bfloat16 else 0


def _map_dtype(m):
    return torch.bfloat16 if getattr(m, "map_bf16", False) else torch.float32


def _conv_bf16(m, xmap, Cout, k):
    if not getattr(m, "conv_bf16", False) or xmap.sc != 1 or (xmap.sn | xmap.sh | xmap.sw) % 4 or xmap.p() % 16:
        return False
    return bool(_lib.load().es_conv2d_bf16_eligible(xmap.C, Cout, k, k))


class _GradSink:
    """The gradient of a map with two consumers summed in place instead of by autograd's add (a full
    extra read-read-write pass over the map): a ConvBlock's input feeds conv1 and the residual
    (identity into bn3, or residual_conv).  (Its x2, which feeds conv3 and the transformer branch's
    FCUDown on the branch stream, keeps autograd's add: the cross-stream wait cost what the add
    saved, S1 195.5 vs 194.7 ms.)  The first consumer's backward writes the buffer (take -> a
    fresh map, accumulate 0) and returns None for the map (give); the second waits for the first's
    event, accumulates into the buffer (the data-gradient kernels' accumulate mode) and returns it.
    bn3's backward always runs before conv1's (conv1's output gradient depends on it)."""
    __slots__ = ("buf", "ev")

    def __init__(self):
        self.buf, self.ev = None, None

    def take(self, alloc):
        """(dx buffer, accumulate flag) for the consumer whose backward runs now; alloc() makes the
        buffer when it is the first."""
        if self.buf is None:
            return alloc(), 0
        cur = torch.cuda.current_stream(self.buf.device)
        cur.wait_event(self.ev)
        self.buf.record_stream(cur)
        return self.buf, 1

    def give(self, dx, acc):
        """What the backward returns for the map after writing dx (acc as take returned it)."""
        if acc:
            self.buf, self.ev = None, None
            return dx
        self.buf, self.ev = dx, torch.cuda.Event()
        self.ev.record(torch.cuda.current_stream(dx.device))
        return None


# test hook (tests/test_gpu_s1_blocks.py, teacher-forced per-op parity of the transformer branch at S1's
# shape): called as BLOCK_CAPTURE("fwd", prefix, n, xt, h1, qkv, o, lse, xmid, h2, gd, act, out) after a
# transformer block's forward with gradients (gd = GELU'(fc1 pre-activation)) and BLOCK_CAPTURE("bwd",
# prefix, n, dout, dxb, dpre, dh, dxm, dxmb, do, dqkv, dh2, dx) after its reverse pass (before the side-stream
# weight gradients are joined), on the launch stream with the block's own buffers; the callee clones what it
# keeps.
BLOCK_CAPTURE = None

# test hook (tests/test_gpu_convs.py, teacher-forced per-conv parity): called as CAPTURE("fwd", wname, x, y,
# spec) after each convolution's forward and CAPTURE("bwd", wname, dy, dx_before, dx) after its input
# gradient, on the launch stream, with the conv's own NHWC views (x: the input map as the kernel reads it;
# dx_before: what a gradient sink's buffer held before this conv accumulated into it, else None); the callee
# clones what it keeps.  spec = (bias name, Cout, k, stride, padding, bf16 kernels?)
CAPTURE = None


def _map_view(t, xm):
    return torch.as_strided(t, (xm.N, xm.H, xm.W, xm.C), (xm.sn, xm.sh, xm.sw, xm.sc), xm.off)


class _ConvFn(torch.autograd.Function):
    """Conv2d (groups 1, optional bias) on an NHWC view -> new NHWC map (code/models/conformer.py
    ConvBlock / FCU convs, Conformer.conv1)."""

    @staticmethod
    def forward(ctx, x, m, xmap, wname, bname, Cout, k, s, p, anchor=None, stats=False, sink=None, out_dtype=None):
        Ho, Wo = (xmap.H + 2 * p - k) // s + 1, (xmap.W + 2 * p - k) // s + 1
        y = torch.empty(xmap.N, Ho, Wo, Cout, dtype=out_dtype or torch.float32, device=x.device)
        b16 = _conv_bf16(m, xmap, Cout, k)
        if not b16 and (x.dtype != torch.float32 or y.dtype != torch.float32):
            raise _lib.EndosslCallError(f"{wname}: bf16 maps need the bf16 conv kernels (channel counts % 32)")
        flags = _fl(x) | (_fl(y) << 1)
        args = (xmap.p(), xmap.N, xmap.H, xmap.W, xmap.C, xmap.sn, xmap.sh, xmap.sw, xmap.sc)
        tail = (ptr(m.pview(bname)) if bname else None, Cout, k, k, s, p, ptr(y), Ho * Wo * Cout, Wo * Cout, Cout, 0)
        if b16 and stats and m.training and BN_STATS_FUSED and not (getattr(m, "sync_bn", True)
                                                                    and dist.world_size() > 1):
            # the BatchNorm that follows takes its batch statistics from these per-block partials (one
            # rank's rows only: a SyncBatchNorm at N > 1 sums global statistics itself, _BNFn, so the
            # partials are requested only when they will be consumed)
            lib = _lib.load()
            part = torch.empty(lib.es_conv2d_bnstats_size(xmap.N * Ho * Wo, Cout), device=x.device)
            call("es_conv2d_fwd_bf16_ex", *args, ptr(m.conv_pack(wname, Cout, xmap.C, k)[0]), *tail, ptr(part), flags,
                 _s())
            m._bn_partials[y.data_ptr()] = (part, y.shape)
        elif b16:
            call("es_conv2d_fwd_bf16_ex", *args, ptr(m.conv_pack(wname, Cout, xmap.C, k)[0]), *tail, None, flags, _s())
        else:
            call("es_conv2d_fwd", *args, ptr(m.pview(wname)), *tail, _s())
        ctx.save_for_backward(x)
        ctx.m, ctx.xmap, ctx.spec, ctx.b16 = m, xmap, (wname, bname, Cout, k, s, p, Ho, Wo), b16
        ctx.sink = sink
        if CAPTURE is not None:
            CAPTURE("fwd", wname, _map_view(xmap.t, xmap), y, (bname, Cout, k, s, p, b16))
        return y

    @staticmethod
    def backward(ctx, dy):
        _own(dy)
        (x,) = ctx.saved_tensors
        m, xm = ctx.m, ctx.xmap
        wname, bname, Cout, k, s, p, Ho, Wo = ctx.spec
        dy = dy.contiguous()
        xp = ptr(x) + x.element_size() * xm.off
        M = xm.N * Ho * Wo
        lib = _lib.load()
        b16 = ctx.b16
        if b16:  # the bf16 weight gradient sizes its own pixel split (splits = 0)
            splits, dwfn = 0, "es_conv2d_bwd_weight_bf16_ex"
            wsn = lib.es_conv2d_bwd_weight_bf16_workspace(M, Cout, xm.C, k, k, 0)
        else:  # pixel splits sized for ~2048 workgroups (8 per CU) over es_conv2d_bwd_weight's tiles
            tiles = lib.es_conv2d_dw_tiles(Cout, xm.C, k, k)
            splits, dwfn = max(1, min(-(-M // 64), -(-2048 // tiles))), "es_conv2d_bwd_weight"
            wsn = lib.es_conv2d_bwd_weight_workspace(Cout, xm.C, k, k, splits)
        side = _wgrad_stream(dy.device) if CONV_DW_SIDE and dy.is_cuda else None
        if side is not None:
            main = torch.cuda.current_stream(dy.device)
            side.wait_stream(main)
            _queue_join(main, side)
            x.record_stream(side)
            dy.record_stream(side)
        with torch.cuda.stream(side) if side is not None else _nullctx():
            ws = torch.empty(wsn, device=dy.device)
            call(dwfn, xp, xm.N, xm.H, xm.W, xm.C, xm.sn, xm.sh, xm.sw, xm.sc, ptr(dy),
                 Ho * Wo * Cout, Wo * Cout, Cout, Cout, k, k, s, p, splits, ptr(ws), ptr(m.gview(wname)), 0,
                 *((_fl(x) | (_fl(dy) << 1),) if b16 else ()), _s())
            if bname:
                wsb = torch.empty(lib.es_chan_workspace(M, Cout), device=dy.device)
                call("es_chan_sum_ex", ptr(dy), M, Cout, M * Cout, Cout, M, ptr(wsb), ptr(m.gview(bname)), 0, _fl(dy),
                     _s())
        dx = None
        if ctx.needs_input_grad[0]:
            full = xm.off == 0 and xm.sc == 1 and xm.sn * xm.N == x.numel()
            sink = ctx.sink
            alloc = (lambda: torch.empty_like(x)) if full else (lambda: torch.zeros_like(x))  # noqa: E731
            dx, acc = sink.take(alloc) if sink is not None else (alloc(), 0)
            wimg = m.conv_pack(wname, Cout, xm.C, k)[1] if b16 else m.pview(wname)
            before = _map_view(dx, xm).clone() if CAPTURE is not None and acc else None
            call("es_conv2d_bwd_data_bf16_ex" if b16 else "es_conv2d_bwd_data", ptr(dy), Ho * Wo * Cout, Wo * Cout, Cout,
                 ptr(wimg), xm.N, xm.H, xm.W, xm.C, Cout, k, k, s, p, ptr(dx) + dx.element_size() * xm.off, xm.sn, xm.sh,
                 xm.sw, xm.sc, acc, *((_fl(dy) | (_fl(dx) << 1),) if b16 else ()), _s())
            if CAPTURE is not None:
                CAPTURE("bwd", wname, dy, before, _map_view(dx, xm))
            if sink is not None:  # first consumer: hand the buffer over; second: return the sum
                dx = sink.give(dx, acc)
        elif CAPTURE is not None:  # no input gradient (the stem reads the images): dy for the weight gradient
            CAPTURE("bwd", wname, dy, None, None)
        return dx, None, None, None, None, None, None, None, None, None, None, None, None


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def conv(m, x, xmap, wname, bname, Cout, k, s=1, p=0, anchor=None, stats=False, sink=None, out_dtype=None):
    """stats=True: the output feeds a train-mode BatchNorm, which then takes its batch statistics
    from the conv's epilogue (BN_STATS_FUSED).  sink: a _GradSink shared with x's other consumer.
    out_dtype: the output map's dtype (default: the model's map dtype, _map_dtype)."""
    return _ConvFn.apply(x, m, xmap, wname, bname, Cout, k, s, p, anchor, stats, sink, out_dtype or _map_dtype(m))


class _BNFn(torch.autograd.Function):
    """BatchNorm2d (+ residual) (+ ReLU) on an NHWC map (ConvBlock bn1/bn2/bn3+residual+act3,
    residual_bn, FCUUp bn, Conformer.bn1)."""

    @staticmethod
    def forward(ctx, x, res, m, pre, eps, relu, res_sink=None):
        x = x.contiguous()
        N, H, W, C = x.shape
        rows = N * H * W
        y = torch.empty_like(x)
        train = m.training
        mean = torch.empty(C, device=x.device)
        rstd = torch.empty(C, device=x.device)
        ws = torch.empty(_lib.load().es_chan_workspace(rows, C), device=x.device)
        rm, rv, nbt = m.bn_buffers(pre)
        res_c = res.contiguous() if res is not None else None  # keep temporaries alive across the launch
        world = dist.world_size() if train and getattr(m, "sync_bn", True) else 1
        part = m._bn_partials.pop(x.data_ptr(), None) if train and world == 1 else None
        fl = _fl(x)
        if res_c is not None and res_c.dtype != x.dtype:
            raise _lib.EndosslCallError(f"{pre}: residual map {res_c.dtype} vs input map {x.dtype}")
        if part is not None and part[1] == x.shape:
            call("es_bn2d_fwd_partials_ex", ptr(x), rows, C, ptr(part[0]), ptr(m.pview(pre + "weight")),
                 ptr(m.pview(pre + "bias")), ptr(rm), ptr(rv), ptr(nbt), BN_MOMENTUM, eps, ptr(res_c),
                 1 if relu else 0, ptr(y), ptr(mean), ptr(rstd), fl, _s())
        elif world > 1:
            # SyncBatchNorm over every rank's rows (the single-process statistics)
            rows_g = rows * world
            sums = torch.empty(2, C, device=x.device)
            call("es_bn2d_sums_ex", ptr(x), rows, C, 0, None, 0, ptr(sums[0]), ptr(ws), fl, _s())
            dist.allreduce_inplace_(sums[0])
            call("es_bn2d_sums_ex", ptr(x), rows, C, 1, ptr(sums[0]), rows_g, ptr(sums[1]), ptr(ws), fl, _s())
            dist.allreduce_inplace_(sums[1])
            call("es_bn2d_fwd_global_ex", ptr(x), rows, C, ptr(m.pview(pre + "weight")), ptr(m.pview(pre + "bias")),
                 ptr(rm), ptr(rv), ptr(nbt), BN_MOMENTUM, eps, ptr(sums[0]), ptr(sums[1]), rows_g, ptr(res_c),
                 1 if relu else 0, ptr(y), ptr(mean), ptr(rstd), fl, _s())
        else:
            call("es_bn2d_fwd_ex", ptr(x), rows, C, ptr(m.pview(pre + "weight")), ptr(m.pview(pre + "bias")), ptr(rm),
                 ptr(rv), ptr(nbt) if train else None, BN_MOMENTUM, eps, 1 if train else 0, ptr(res_c),
                 1 if relu else 0, ptr(y), ptr(mean), ptr(rstd), ptr(ws), fl, _s())
        # the ReLU mask of a train-mode BatchNorm without residual is rebuilt from x in the backward
        # (es_bn2d_bwd_recompute_ex): y is not read there (one map read less in both backward kernels)
        keep_y = relu and (res is not None or world > 1 or not train or not BN_Y_FREE)
        ctx.save_for_backward(x, y if keep_y else None, mean, rstd)
        ctx.m, ctx.pre, ctx.eps, ctx.relu, ctx.train, ctx.has_res = m, pre, eps, relu, train, res is not None
        ctx.world = world
        ctx.res_sink = res_sink if res is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        _own(dy)
        x, y, mean, rstd = ctx.saved_tensors
        m, pre = ctx.m, ctx.pre
        N, H, W, C = x.shape
        rows = N * H * W
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        gout = torch.empty_like(x) if ctx.has_res else None
        ws = torch.empty(_lib.load().es_chan_workspace(rows, C), device=x.device)
        _, rv, _ = m.bn_buffers(pre)
        fl = _fl(x)
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        if ctx.world > 1:
            loc = torch.empty(2 * C, device=x.device)
            call("es_bn2d_bwd_sums_ex", ptr(x), ptr(y), ptr(dy), rows, C, 1 if ctx.relu else 0, ptr(mean), ptr(rstd),
                 ptr(loc), ptr(ws), fl, _s())
            glob = dist.allreduce_inplace_(loc.clone())
            call("es_bn2d_bwd_global_ex", ptr(x), ptr(y), ptr(dy), rows, C, 1 if ctx.relu else 0,
                 ptr(m.pview(pre + "weight")), ptr(mean), ptr(rstd), ptr(loc), ptr(glob), rows * ctx.world, ptr(dx),
                 ptr(gout), ptr(m.gview(pre + "weight")), ptr(m.gview(pre + "bias")), 0, fl, _s())
            return dx, _BNFn._res_grad(ctx, gout), None, None, None, None, None
        if ctx.relu and y is None:
            call("es_bn2d_bwd_recompute_ex", ptr(x), ptr(dy), rows, C, ptr(m.pview(pre + "weight")),
                 ptr(m.pview(pre + "bias")), ptr(mean), ptr(rstd), ptr(dx), ptr(m.gview(pre + "weight")),
                 ptr(m.gview(pre + "bias")), 0, ptr(ws), fl, _s())
            return dx, None, None, None, None, None, None
        call("es_bn2d_bwd_ex", ptr(x), ptr(y), ptr(dy), rows, C, 1 if ctx.relu else 0, ptr(m.pview(pre + "weight")),
             ptr(mean), ptr(rstd), 1 if ctx.train else 0, ptr(rv), ctx.eps, ptr(dx), ptr(gout),
             ptr(m.gview(pre + "weight")), ptr(m.gview(pre + "bias")), 0, ptr(ws), fl, _s())
        return dx, _BNFn._res_grad(ctx, gout), None, None, None, None, None

    @staticmethod
    def _res_grad(ctx, gout):
        """The residual's gradient, or None with it handed to the residual map's _GradSink."""
        sink = ctx.res_sink
        if gout is None or sink is None:
            return gout
        if sink.buf is None:
            return sink.give(gout, 0)
        buf, _ = sink.take(None)  # (not reached in the Conformer / ResNet graphs: bn3 runs first)
        buf.add_(gout)
        return sink.give(buf, 1)


def bn(m, x, pre, eps=BN_EPS_BLOCK, relu=False, res=None, res_sink=None):
    return _BNFn.apply(x, res, m, pre, eps, relu, res_sink)


class _BNConvFn(torch.autograd.Function):
    """relu(BatchNorm2d(x)) -> Conv2d with the normalised map never written (code/models/conformer.py:118-134:
    ConvBlock bn1 -> act1 -> conv2, bn2 -> act2 -> conv3).  Forward: the batch statistics from the producing
    conv's epilogue partials (es_bn2d_fwd_partials_ex with y = NULL: running buffers, mean / rstd), then the
    conv gathers relu((x - mean) rstd gamma + beta) rounded to the map's type (es_conv2d_fwd_bf16_bnin_ex) --
    bit for bit the operand bn() would have written.  Backward: the conv's data gradient d(BN output), its
    weight gradient with the same BatchNorm-applying gather (side stream), and the BatchNorm backward that
    rebuilds the ReLU mask from x (es_bn2d_bwd_recompute_ex): every gradient bit-identical to bn() + conv()."""

    @staticmethod
    def forward(ctx, x, m, pre, eps, wname, bname, Cout, k, s, p, stats, out_dtype):
        N, H, W, C = x.shape
        rows = N * H * W
        mean = torch.empty(C, device=x.device)
        rstd = torch.empty(C, device=x.device)
        rm, rv, nbt = m.bn_buffers(pre)
        part = m._bn_partials.pop(x.data_ptr())
        fl = _fl(x)
        gam, bet = m.pview(pre + "weight"), m.pview(pre + "bias")
        call("es_bn2d_fwd_partials_ex", ptr(x), rows, C, ptr(part[0]), ptr(gam), ptr(bet), ptr(rm), ptr(rv), ptr(nbt),
             BN_MOMENTUM, eps, None, 1, None, ptr(mean), ptr(rstd), fl, _s())
        xmap = _Map.nhwc(x)
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y = torch.empty(N, Ho, Wo, Cout, dtype=out_dtype, device=x.device)
        flags = fl | (_fl(y) << 1)
        args = (xmap.p(), N, H, W, C, xmap.sn, xmap.sh, xmap.sw, xmap.sc)
        tail = (ptr(m.pview(bname)) if bname else None, Cout, k, k, s, p, ptr(y), Ho * Wo * Cout, Wo * Cout, Cout, 0)
        part_out = None
        if stats and BN_STATS_FUSED:  # the next BatchNorm's statistics, as _ConvFn (train mode, world 1 here)
            part_out = torch.empty(_lib.load().es_conv2d_bnstats_size(N * Ho * Wo, Cout), device=x.device)
        call("es_conv2d_fwd_bf16_bnin_ex", *args, ptr(m.conv_pack(wname, Cout, C, k)[0]), *tail,
             ptr(part_out) if part_out is not None else None, flags, ptr(mean), ptr(rstd), ptr(gam), ptr(bet), _s())
        if part_out is not None:
            m._bn_partials[y.data_ptr()] = (part_out, y.shape)
        ctx.save_for_backward(x, mean, rstd)
        ctx.m, ctx.pre, ctx.spec = m, pre, (wname, bname, Cout, k, s, p, Ho, Wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        _own(dy)
        x, mean, rstd = ctx.saved_tensors
        m, pre = ctx.m, ctx.pre
        wname, bname, Cout, k, s, p, Ho, Wo = ctx.spec
        N, H, W, C = x.shape
        rows, M = N * H * W, N * Ho * Wo
        dy = dy.contiguous()
        lib = _lib.load()
        gam, bet = m.pview(pre + "weight"), m.pview(pre + "bias")
        side = _wgrad_stream(dy.device) if CONV_DW_SIDE and dy.is_cuda else None
        if side is not None:
            main = torch.cuda.current_stream(dy.device)
            side.wait_stream(main)
            _queue_join(main, side)
            for t in (x, dy, mean, rstd):
                t.record_stream(side)
        with torch.cuda.stream(side) if side is not None else _nullctx():
            ws = torch.empty(lib.es_conv2d_bwd_weight_bf16_workspace(M, Cout, C, k, k, 0), device=dy.device)
            call("es_conv2d_bwd_weight_bf16_bnin_ex", ptr(x), N, H, W, C, H * W * C, W * C, C, 1, ptr(dy),
                 Ho * Wo * Cout, Wo * Cout, Cout, Cout, k, k, s, p, 0, ptr(ws), ptr(m.gview(wname)), 0,
                 _fl(x) | (_fl(dy) << 1), ptr(mean), ptr(rstd), ptr(gam), ptr(bet), _s())
            if bname:
                wsb = torch.empty(lib.es_chan_workspace(M, Cout), device=dy.device)
                call("es_chan_sum_ex", ptr(dy), M, Cout, M * Cout, Cout, M, ptr(wsb), ptr(m.gview(bname)), 0, _fl(dy),
                     _s())
        dh = torch.empty_like(x)  # d(loss) / d(BN output): every pixel written (all stride phases)
        call("es_conv2d_bwd_data_bf16_ex", ptr(dy), Ho * Wo * Cout, Wo * Cout, Cout, ptr(m.conv_pack(wname, Cout, C, k)[1]),
             N, H, W, C, Cout, k, k, s, p, ptr(dh), H * W * C, W * C, C, 1, 0, _fl(dy) | (_fl(dh) << 1), _s())
        dx = torch.empty_like(x)
        wsn = torch.empty(lib.es_chan_workspace(rows, C), device=x.device)
        call("es_bn2d_bwd_recompute_ex", ptr(x), ptr(dh), rows, C, ptr(gam), ptr(bet), ptr(mean), ptr(rstd), ptr(dx),
             ptr(m.gview(pre + "weight")), ptr(m.gview(pre + "bias")), 0, ptr(wsn), _fl(x), _s())
        return dx, None, None, None, None, None, None, None, None, None, None, None


def bn_conv(m, x, pre, wname, bname, Cout, k, s=1, p=0, stats=False, out_dtype=None, eps=BN_EPS_BLOCK):
    """conv(relu(bn(x))) for a train-mode BatchNorm whose output feeds this conv alone: fused (_BNConvFn) when the
    conv runs on the bf16 kernels and the BatchNorm takes its statistics from x's producing conv (one rank's
    rows); otherwise the two ops with the normalised map in between."""
    out_dtype = out_dtype or _map_dtype(m)
    world = dist.world_size() if getattr(m, "sync_bn", True) else 1
    part = m._bn_partials.get(x.data_ptr())
    if (BN_CONV_FUSED and (k == 1 or BN_CONV_FUSED_KXK) and BN_Y_FREE and m.training and world == 1
            and CAPTURE is None and part is not None
            and part[1] == x.shape and x.is_contiguous() and _conv_bf16(m, _Map.nhwc(x), Cout, k)):
        return _BNConvFn.apply(x, m, pre, eps, wname, bname, Cout, k, s, p, stats, out_dtype)
    h = bn(m, x, pre, eps=eps, relu=True)
    return conv(m, h, _Map.nhwc(h), wname, bname, Cout, k, s, p, stats=stats, out_dtype=out_dtype)


class _MaxPoolFn(torch.autograd.Function):
    """MaxPool2d on the stem's fp32 map; out_dtype bf16: the pooled map starts the bf16 maps."""

    @staticmethod
    def forward(ctx, x, k, s, p, out_dtype=None):
        N, H, W, C = x.shape
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y = torch.empty(N, Ho, Wo, C, dtype=out_dtype or torch.float32, device=x.device)
        arg = torch.empty(N, Ho, Wo, C, dtype=torch.int8, device=x.device)
        call("es_maxpool2d_fwd_ex", ptr(x), N, H, W, C, k, s, p, ptr(y), ptr(arg), _fl(y) << 1, _s())
        ctx.save_for_backward(arg)
        ctx.geom = (N, H, W, C, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        _own(dy)
        (arg,) = ctx.saved_tensors
        N, H, W, C, k, s, p = ctx.geom
        dx = torch.empty(N, H, W, C, device=dy.device)
        dy = dy.contiguous()
        call("es_maxpool2d_bwd_ex", ptr(dy), ptr(arg), N, H, W, C, k, s, p, ptr(dx), _fl(dy), _s())
        return dx, None, None, None, None


class _AvgPoolFn(torch.autograd.Function):
    """AvgPool2d(k, k) map -> map of the same dtype."""

    @staticmethod
    def forward(ctx, x, k):
        N, H, W, C = x.shape
        y = torch.empty(N, H // k, W // k, C, dtype=x.dtype, device=x.device)
        call("es_avgpool2d_fwd_ex", ptr(x.contiguous()), N, H, W, C, k, ptr(y), _fl(x) | (_fl(y) << 1), _s())
        ctx.geom, ctx.dt = (N, H, W, C, k), x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        _own(dy)
        N, H, W, C, k = ctx.geom
        dx = torch.empty(N, H, W, C, dtype=ctx.dt, device=dy.device)
        dy = dy.contiguous()
        call("es_avgpool2d_bwd_ex", ptr(dy), N, H, W, C, k, ptr(dx), 0, _fl(dy) | (_fl(dx) << 1), _s())
        return dx, None


class _UpsampleAddFn(torch.autograd.Function):
    """base + F.interpolate(src, nearest, x s)  (FCUUp output added before conv2, :120,194)."""

    @staticmethod
    def forward(ctx, base, src, s):
        N, H, W, C = base.shape
        out = torch.empty_like(base)
        base_c, src_c = base.contiguous(), src.contiguous()
        if src_c.dtype != base_c.dtype:
            raise _lib.EndosslCallError(f"upsample-add of a {src_c.dtype} map onto a {base_c.dtype} map")
        call("es_upsample_add_fwd_ex", ptr(base_c), ptr(src_c), N, H, W, C, s, ptr(out), _fl(base_c), _s())
        ctx.geom = (N, H, W, C, s)
        return out

    @staticmethod
    def backward(ctx, dout):
        _own(dout)
        N, H, W, C, s = ctx.geom
        dout = dout.contiguous()
        dsrc = torch.empty(N, H // s, W // s, C, dtype=dout.dtype, device=dout.device)
        call("es_upsample_bwd_ex", ptr(dout), N, H, W, C, s, ptr(dsrc), _fl(dout), _s())
        return dout, dsrc, None


class _FcuTokensFn(torch.autograd.Function):
    """FCUDown's LayerNorm + GELU + cat(cls) fused with ConvTransBlock's `x_st + x_t`."""

    @staticmethod
    def forward(ctx, pooled, xt, m, pre, sink=None):
        N, h, w, D = pooled.shape
        np_ = h * w
        out = _zero_pad(torch.empty_like(xt), N * (np_ + 1))  # the kernel writes every token row
        mean = torch.empty(N * np_, device=xt.device)
        rstd = torch.empty(N * np_, device=xt.device)
        call("es_fcu_down_tokens_fwd", ptr(pooled.contiguous()), ptr(xt), ptr(m.pview(pre + "ln.weight")),
             ptr(m.pview(pre + "ln.bias")), ptr(out), ptr(mean), ptr(rstd), N, np_, D, LN_EPS, _s())
        ctx.save_for_backward(pooled, mean, rstd)
        ctx.m, ctx.pre, ctx.sink = m, pre, sink
        return out

    @staticmethod
    def backward(ctx, dout):
        _own(dout)
        pooled, mean, rstd = ctx.saved_tensors
        m, pre = ctx.m, ctx.pre
        N, h, w, D = pooled.shape
        np_ = h * w
        dout = dout.contiguous()
        alloc = lambda: _zero_pad(torch.empty_like(dout), N * (np_ + 1))  # noqa: E731
        sink = ctx.sink
        dxt, acc = sink.take(alloc) if sink is not None else (alloc(), 0)
        dpooled = torch.empty_like(pooled)
        ws = torch.empty(_lib.load().es_fcu_down_workspace(N, np_, D), device=dout.device)
        call("es_fcu_down_tokens_bwd_ex", ptr(dout), ptr(pooled), ptr(m.pview(pre + "ln.weight")),
             ptr(m.pview(pre + "ln.bias")), ptr(mean), ptr(rstd), ptr(dxt), ptr(dpooled),
             ptr(m.gview(pre + "ln.weight")), ptr(m.gview(pre + "ln.bias")), 0, N, np_, D, ptr(ws), acc, _s())
        if sink is not None:
            dxt = sink.give(dxt, acc)
        return dpooled, dxt, None, None, None


class _PatchTokensFn(torch.autograd.Function):
    """trans_patch_conv (k = s = patch/4) into token rows 1.., cls_token into row 0
    (Conformer.forward :426-428; no position embedding)."""

    @staticmethod
    def forward(ctx, xb, m):
        cfg = m.cfg
        N, H, W, C = xb.shape
        D, T, g, dw = cfg.dim, cfg.T, cfg.grid, cfg.dw
        xt = torch.zeros(_rup(N * T, 256), D, device=xb.device)
        b16 = _conv_bf16(m, _Map.nhwc(xb), D, dw)
        wimg = m.conv_pack("trans_patch_conv.weight", D, C, dw)[0] if b16 else m.pview("trans_patch_conv.weight")
        if not b16 and xb.dtype != torch.float32:
            raise _lib.EndosslCallError("trans_patch_conv: a bf16 map needs the bf16 conv kernels")
        call("es_conv2d_fwd_bf16_ex" if b16 else "es_conv2d_fwd", ptr(xb), N, H, W, C, H * W * C, W * C, C, 1, ptr(wimg),
             ptr(m.pview("trans_patch_conv.bias")), D, dw, dw, dw, 0, ptr(xt) + 4 * D, T * D, g * D, D, 0,
             *((None, _fl(xb)) if b16 else ()), _s())
        call("es_tokens_cls_set", ptr(xt), N, T, D, ptr(m.pview("cls_token")), _s())
        ctx.save_for_backward(xb)
        ctx.m, ctx.b16 = m, b16
        return xt

    @staticmethod
    def backward(ctx, dxt):
        _own(dxt)
        (xb,) = ctx.saved_tensors
        m = ctx.m
        cfg = m.cfg
        N, H, W, C = xb.shape
        D, T, g, dw = cfg.dim, cfg.T, cfg.grid, cfg.dw
        dxt = dxt.contiguous()
        lib = _lib.load()
        M = N * cfg.np
        b16 = ctx.b16
        if b16:
            splits = 0
            ws = torch.empty(lib.es_conv2d_bwd_weight_bf16_workspace(M, D, C, dw, dw, 0), device=dxt.device)
        else:
            splits = max(1, min(-(-M // 64), -(-2048 // lib.es_conv2d_dw_tiles(D, C, dw, dw))))
            ws = torch.empty(lib.es_conv2d_bwd_weight_workspace(D, C, dw, dw, splits), device=dxt.device)
        dyp = ptr(dxt) + 4 * D
        call("es_conv2d_bwd_weight_bf16_ex" if b16 else "es_conv2d_bwd_weight", ptr(xb), N, H, W, C, H * W * C, W * C, C,
             1, dyp, T * D, g * D, D, D, dw, dw, dw, 0, splits, ptr(ws), ptr(m.gview("trans_patch_conv.weight")), 0,
             *((_fl(xb),) if b16 else ()), _s())
        wsb = torch.empty(lib.es_chan_workspace(M, D), device=dxt.device)
        call("es_chan_sum", dyp, M, D, T * D, D, cfg.np, ptr(wsb), ptr(m.gview("trans_patch_conv.bias")), 0, _s())
        call("es_chan_sum", ptr(dxt), N, D, T * D, 0, 1, ptr(wsb), ptr(m.gview("cls_token")), 0, _s())
        dxb = torch.empty_like(xb)
        wimg = m.conv_pack("trans_patch_conv.weight", D, C, dw)[1] if b16 else m.pview("trans_patch_conv.weight")
        call("es_conv2d_bwd_data_bf16_ex" if b16 else "es_conv2d_bwd_data", dyp, T * D, g * D, D, ptr(wimg), N, H, W, C,
             D, dw, dw, dw, 0, ptr(dxb), H * W * C, W * C, C, 1, 0, *((_fl(dxb) << 1,) if b16 else ()), _s())
        return dxb, None


class _BlockFn(torch.autograd.Function):
    """conformer.Block (code/models/conformer.py:55-72) on the padded token buffer [Mp, D]: bf16
    MFMA GEMMs, fused attention, LayerNorm kernels (the ViT engine's launch sequence)."""

    @staticmethod
    def forward(ctx, xt, m, pre):
        cfg = m.cfg
        D, Hd, T, H = cfg.dim, cfg.hidden, cfg.T, cfg.heads
        Mp = xt.shape[0]
        n = m.cur_n
        M = n * T
        s = _s()
        dev = xt.device
        b16 = torch.bfloat16
        # rows [M, Mp) of the weight-gradient GEMM operands (h1, o, h2, act) must read as zero; every
        # other buffer is read on its first M rows only, so it needs no fill at all
        e = lambda *sh, dt=torch.float32: torch.empty(*sh, dtype=dt, device=dev)  # noqa: E731
        zp = lambda *sh, dt=torch.float32: _zero_pad(e(*sh, dt=dt), M)  # noqa: E731
        h1, h2 = zp(Mp, D, dt=b16), zp(Mp, D, dt=b16)
        mean1, rstd1, mean2, rstd2 = e(Mp), e(Mp), e(Mp), e(Mp)
        qkv, o = e(Mp, 3 * D, dt=b16), zp(Mp, D, dt=b16)
        lse = e(n * H * T)
        xmid, out = e(Mp, D), zp(Mp, D)
        # fc1 + GELU: with gradients the epilogue writes GELU'(pre) beside the activation (the ViT engine's
        # GELU_D form), so the backward's fc2 data gradient multiplies by it (EPI_MULAUX) instead of
        # re-evaluating the erf per element behind its K loop (EPI_DGELU: 1.6 ms per S1 launch); without
        # gradients (the weak pass) the activation alone
        grad = ctx.needs_input_grad[0]
        gd, act = (e(Mp, Hd, dt=b16) if grad else None), zp(Mp, Hd, dt=b16)
        pv, wb = m.pview, m.wb
        call("es_layernorm_fwd", ptr(xt), D, ptr(pv(pre + "norm1.weight")), ptr(pv(pre + "norm1.bias")), ptr(h1), D,
             ptr(mean1), ptr(rstd1), M, D, LN_EPS, s)
        call("es_gemm_nt", EPI_BF16, ptr(h1), D, ptr(wb[pre + "attn.qkv.weight"]), D, ptr(pv(pre + "attn.qkv.bias")),
             ptr(qkv), 3 * D, None, None, 0, M, 3 * D, D, 0, s)
        call("es_attn_fwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), n, T, H, 64 ** -0.5, s)
        call("es_gemm_nt", EPI_F32_RESID, ptr(o), D, ptr(wb[pre + "attn.proj.weight"]), D,
             ptr(pv(pre + "attn.proj.bias")), ptr(xmid), D, None, ptr(xt), D, M, D, D, 0, s)
        call("es_layernorm_fwd", ptr(xmid), D, ptr(pv(pre + "norm2.weight")), ptr(pv(pre + "norm2.bias")), ptr(h2), D,
             ptr(mean2), ptr(rstd2), M, D, LN_EPS, s)
        if grad:
            call("es_gemm_nt", EPI_GELU_D, ptr(h2), D, ptr(wb[pre + "mlp.fc1.weight"]), D,
                 ptr(pv(pre + "mlp.fc1.bias")), ptr(gd), Hd, ptr(act), None, 0, M, Hd, D, 0, s)
        else:
            call("es_gemm_nt", EPI_GELU_ACT, ptr(h2), D, ptr(wb[pre + "mlp.fc1.weight"]), D,
                 ptr(pv(pre + "mlp.fc1.bias")), ptr(act), Hd, None, None, 0, M, Hd, D, 0, s)
        call("es_gemm_nt", EPI_F32_RESID, ptr(act), Hd, ptr(wb[pre + "mlp.fc2.weight"]), Hd,
             ptr(pv(pre + "mlp.fc2.bias")), ptr(out), D, None, ptr(xmid), D, M, D, Hd, 0, s)
        ctx.save_for_backward(xt, h1, mean1, rstd1, qkv, o, lse, xmid, h2, mean2, rstd2, gd, act)
        ctx.m, ctx.pre, ctx.n = m, pre, n
        if BLOCK_CAPTURE is not None and grad:
            BLOCK_CAPTURE("fwd", pre, n, xt, h1, qkv, o, lse, xmid, h2, gd, act, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        _own(dout)
        xt, h1, mean1, rstd1, qkv, o, lse, xmid, h2, mean2, rstd2, gd, act = ctx.saved_tensors
        m, pre, n = ctx.m, ctx.pre, ctx.n
        cfg = m.cfg
        D, Hd, T, H = cfg.dim, cfg.hidden, cfg.T, cfg.heads
        Mp = xt.shape[0]
        M = n * T
        s = _s()
        dev = xt.device
        b16 = torch.bfloat16
        # layer-internal scratch, reused by every other block's backward: allocated zeroed once, so the
        # pad rows the weight-gradient GEMMs read stay zero.  Two sets alternate by block, because the
        # weight gradients (side stream, CONV_DW_SIDE) of the block before may still be reading its set;
        # this block waits for the side-stream event of the last block that used its set.
        side = _wgrad_stream(dev) if CONV_DW_SIDE and xt.is_cuda else None
        main = torch.cuda.current_stream(dev) if xt.is_cuda else None
        k = m._blk_set = getattr(m, "_blk_set", 0) ^ 1
        z = lambda name, *sh, dt=torch.float32: m.bwd_scratch(f"{name}/{k}", sh, dt)  # noqa: E731
        if not hasattr(m, "_blk_events"):
            m._blk_events = {}
        if side is not None and k in m._blk_events:
            main.wait_event(m._blk_events.pop(k))
        lib = _lib.load()
        dout = dout.contiguous()
        dxb = z("dxb", Mp, D, dt=b16)
        call("es_cast_f32_bf16", ptr(dout), ptr(dxb), Mp * D, s)
        wt, pv, gv = m.wt, m.pview, m.gview
        ws_ln = torch.empty(2 * 1024 * D, device=dev)

        # the grouped launch's shapes: every N1 a multiple of 384, every N2 of 192; rows [M, Mp) of every
        # operand zero (h1 / o / h2 / act zero-padded in the forward, the dy scratch zeroed once), Mp >= M + 63
        grouped = (CONF_TN_GROUPED and xt.is_cuda and D % 384 == 0 and Hd % 384 == 0 and Mp >= _rup(M, 64))
        probs = []

        def wgrad(dy, N1, x, N2, wname, bname):
            if grouped:
                probs.append((dy, N1, x, N2, wname, bname))
                return
            sp = _tn_splits(M, N1, N2)
            if side is not None and CONF_TN_SHARE < 1.0 and M >= 65536 and N1 % 384 == 0 and N2 % 192 == 0:
                # beside the branch streams: the 384 x 192 tile on a share of the CUs (as Engine.TN_SHARE)
                ncu = torch.cuda.get_device_properties(dev).multi_processor_count
                sp = max(1, int(ncu * CONF_TN_SHARE) // ((N1 // 384) * (N2 // 192)))
            if side is not None:
                side.wait_stream(main)
            with torch.cuda.stream(side) if side is not None else _nullctx():
                ws = torch.empty(lib.es_gemm_tn_workspace(N1, N2, sp), device=dev)
                call("es_gemm_tn", ptr(dy), N1, ptr(x), N2, M, N1, N2, sp, ptr(ws), ptr(gv(wname)), 0,
                     ptr(gv(bname)), _s())

        dpre = z("dpre", Mp, Hd, dt=b16)
        call("es_gemm_nt", EPI_MULAUX, ptr(dxb), D, ptr(wt[pre + "mlp.fc2.weight"]), D, None, ptr(dpre), Hd, None,
             ptr(gd), Hd, M, Hd, D, 0, s)
        wgrad(dxb, D, act, Hd, pre + "mlp.fc2.weight", pre + "mlp.fc2.bias")
        dh = z("dh", Mp, D, dt=b16)  # d(LN output) in bf16, as the ViT engine (Engine.DH_BF16)
        call("es_gemm_nt", EPI_BF16, ptr(dpre), Hd, ptr(wt[pre + "mlp.fc1.weight"]), Hd, None, ptr(dh), D, None,
             None, 0, M, D, Hd, 0, s)
        wgrad(dpre, Hd, h2, D, pre + "mlp.fc1.weight", pre + "mlp.fc1.bias")
        dxm, dxmb = z("dxm", Mp, D), z("dxmb", Mp, D, dt=b16)
        call("es_layernorm_bwd_b16", ptr(dh), D, ptr(xmid), D, ptr(mean2), ptr(rstd2), ptr(pv(pre + "norm2.weight")),
             ptr(dout), D, ptr(dxm), D, ptr(dxmb), D, ptr(gv(pre + "norm2.weight")), ptr(gv(pre + "norm2.bias")),
             ptr(ws_ln), 1024, M, D, 0, s)
        do = z("do", Mp, D, dt=b16)
        call("es_gemm_nt", EPI_BF16, ptr(dxmb), D, ptr(wt[pre + "attn.proj.weight"]), D, None, ptr(do), D, None,
             None, 0, M, D, D, 0, s)
        wgrad(dxmb, D, o, D, pre + "attn.proj.weight", pre + "attn.proj.bias")
        dqkv = z("dqkv", Mp, 3 * D, dt=b16)
        delta = z("delta", n * H * T)
        call("es_attn_bwd", ptr(qkv), 3 * D, ptr(o), D, ptr(lse), ptr(delta), ptr(do), D, ptr(dqkv), 3 * D, n, T, H,
             64 ** -0.5, s)
        dh2 = z("dh2", Mp, D, dt=b16)
        call("es_gemm_nt", EPI_BF16, ptr(dqkv), 3 * D, ptr(wt[pre + "attn.qkv.weight"]), 3 * D, None, ptr(dh2), D,
             None, None, 0, M, D, 3 * D, 0, s)
        wgrad(dqkv, 3 * D, h1, D, pre + "attn.qkv.weight", pre + "attn.qkv.bias")
        if probs:
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            target = max(1, int(ncu * CONF_TN_SHARE)) if side is not None else ncu
            if side is not None:
                side.wait_stream(main)
            with torch.cuda.stream(side) if side is not None else _nullctx():
                _wgrad_grouped(m, probs, M, target, k)
        dx = _zero_pad(torch.empty(Mp, D, device=dev), M)  # returned to autograd: fresh
        call("es_layernorm_bwd_b16", ptr(dh2), D, ptr(xt), D, ptr(mean1), ptr(rstd1), ptr(pv(pre + "norm1.weight")),
             ptr(dxm), D, ptr(dx), D, None, 0, ptr(gv(pre + "norm1.weight")), ptr(gv(pre + "norm1.bias")),
             ptr(ws_ln), 1024, M, D, 0, s)
        if BLOCK_CAPTURE is not None:
            BLOCK_CAPTURE("bwd", pre, n, dout, dxb, dpre, dh, dxm, dxmb, do, dqkv, dh2, dx)
        if side is not None:
            for t in (act, h2, o, h1):  # saved activations the side stream still reads
                t.record_stream(side)
            m._blk_events[k] = side.record_event()
            _queue_join(main, side)
        return dx, None, None


class _ConvHeadFn(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) + flatten + conv_cls_head Linear (Conformer.forward :438-439; also
    ResNet's global pool + fc, pre="fc.")."""

    @staticmethod
    def forward(ctx, x, m, anchor=None, pre="conv_cls_head."):
        N, H, W, C = x.shape
        if H != W:
            raise ValueError(f"the global-pool head expects square maps, got {H}x{W}")
        ncls = m.cfg.num_classes
        pooled = torch.empty(N, C, device=x.device)
        call("es_avgpool2d_fwd_ex", ptr(x.contiguous()), N, H, W, C, H, ptr(pooled), _fl(x), _s())
        logits = torch.empty(N, ncls, device=x.device)
        call("es_dense_fwd", ptr(pooled), C, ptr(m.pview(pre + "weight")), ptr(m.pview(pre + "bias")),
             ptr(logits), ncls, N, C, ncls, 0, 0.0, None, 1.0, _s())
        ctx.save_for_backward(pooled)
        ctx.m, ctx.geom, ctx.pre, ctx.dt = m, (N, H, W, C), pre, x.dtype
        return logits

    @staticmethod
    def backward(ctx, dl):
        _own(dl)
        (pooled,) = ctx.saved_tensors
        m = ctx.m
        N, H, W, C = ctx.geom
        ncls = m.cfg.num_classes
        dl = dl.contiguous()
        dpooled = torch.empty(N, C, device=dl.device)
        ws = torch.empty(_lib.load().es_dense_bwd_workspace(N, ncls), device=dl.device)
        pre = ctx.pre
        call("es_dense_bwd", ptr(dl), ncls, None, 0, 0, 0.0, None, 1.0, ptr(pooled), C,
             ptr(m.pview(pre + "weight")), ptr(dpooled), C, 0, ptr(m.gview(pre + "weight")),
             ptr(m.gview(pre + "bias")), N, C, ncls, ptr(ws), _s())
        if getattr(m, "frozen_trunk", False):  # IS_FREEZE: the head's parameters only
            return None, None, None, None
        dx = torch.empty(N, H, W, C, dtype=ctx.dt, device=dl.device)
        call("es_avgpool2d_bwd_ex", ptr(dpooled), N, H, W, C, H, ptr(dx), 0, _fl(dx) << 1, _s())
        return dx, None, None, None


class _TransHeadFn(torch.autograd.Function):
    """trans_norm (LayerNorm eps 1e-5) + trans_cls_head on the CLS token (Conformer.forward :441-443)."""

    @staticmethod
    def forward(ctx, xt, m, anchor=None):
        cfg = m.cfg
        n, D, ncls = m.cur_n, cfg.dim, cfg.num_classes
        logits = torch.empty(n, ncls, device=xt.device)
        xhat = torch.empty(n, D, device=xt.device)
        rstd = torch.empty(n, device=xt.device)
        call("es_cls_head_fwd", ptr(xt), D, cfg.T, ptr(m.pview("trans_norm.weight")), ptr(m.pview("trans_norm.bias")),
             ptr(m.pview("trans_cls_head.weight")), ptr(m.pview("trans_cls_head.bias")), ptr(logits), ncls,
             ptr(xhat), ptr(rstd), n, D, ncls, LN_EPS_TRANS_NORM, _s())
        ctx.save_for_backward(xhat, rstd)
        ctx.m, ctx.n, ctx.Mp = m, n, xt.shape[0]
        return logits

    @staticmethod
    def backward(ctx, dl):
        _own(dl)
        xhat, rstd = ctx.saved_tensors
        m, n = ctx.m, ctx.n
        cfg = m.cfg
        D, ncls = cfg.dim, cfg.num_classes
        frozen = getattr(m, "frozen_trunk", False)  # IS_FREEZE: trans_norm frozen, no input gradient
        dx = torch.zeros(ctx.Mp if not frozen else n, D, device=dl.device)
        dyn = torch.empty(n, D, device=dl.device)
        gn = (m.gview("trans_norm.weight"), m.gview("trans_norm.bias")) if not frozen else \
            (torch.zeros(D, device=dl.device), torch.zeros(D, device=dl.device))
        call("es_cls_head_bwd", ptr(dl.contiguous()), ncls, ptr(m.pview("trans_cls_head.weight")),
             ptr(m.pview("trans_norm.weight")), ptr(m.pview("trans_norm.bias")), ptr(xhat), ptr(rstd), ptr(dyn),
             ptr(dx), D, cfg.T if not frozen else 1, ptr(m.gview("trans_cls_head.weight")),
             ptr(m.gview("trans_cls_head.bias")), ptr(gn[0]), ptr(gn[1]), n, D, ncls, _s())
        return (dx if not frozen else None), None, None


# ------------------------------------------------------------------------------------ model
class NativeConformer(nn.Module):
    """Conformer whose compute runs in libendossl_hip.so; state_dict identical to the reference's."""

    def __init__(self, cfg=None, seed=None, **kw):
        super().__init__()
        self.cfg = cfg if cfg is not None else ConformerConfig(**kw)
        self.layout = conformer_layout(self.cfg)
        self.offs, o = {}, 0
        for name, shape, kind in self.layout:
            if kind == "p":
                self.offs[name] = o
                o = _rup(o + math.prod(shape), 64)
        self.numel = o
        self.shapes = {name: shape for name, shape, _ in self.layout}
        flat = torch.zeros(self.numel, dtype=torch.float32)
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        init_conformer_(flat, self.layout, self.offs, generator=gen)
        self._build(flat, device=torch.device("cpu"))
        self.version = 0
        self.cur_n = 0
        self.conv_bf16 = CONV_BF16

    @property
    def map_bf16(self):
        """bf16 activation / gradient maps after the stem: the bf16 convs on and every conv of the CNN
        branch eligible for them (stage-1 bottleneck s1 / 4 a multiple of 32: Conformer-B's 64)."""
        return bool(self.conv_bf16 and MAP_BF16 and (self.cfg.s1 // 4) % 32 == 0 and self.cfg.s1 % 32 == 0)

    def set_conv_precision(self, precision):
        """"bf16": convs with channel counts % 32 == 0 on bf16 operands (default); "fp32": all on
        conv.hip's fp32 MFMA kernels (the parity mode of the CNN branch)."""
        if precision not in ("bf16", "fp32"):
            raise ValueError(precision)
        self.conv_bf16 = precision == "bf16"
        return self

    def conv_pack(self, name, Cout, Cin, k):
        """bf16 images of conv weight `name` -- wp [Cout][k k][Cin] and wt [Cin][k k][Cout] -- packed
        once per parameter version.  The first step packs each weight at its first use (es_conv2d_pack_bf16)
        and records the model's conv weights; every later version packs them all in one launch
        (es_conv2d_pack_bf16_multi) at the first conv_pack of the version -- the stem, on the caller's
        stream: a conv on another stream waits for that launch's event."""
        ent = self._cpack.get(name)
        if ent is None:
            n = Cout * Cin * k * k
            ent = self._cpack[name] = [-1, torch.empty(n, dtype=torch.bfloat16, device=self.flat.device),
                                       torch.empty(n, dtype=torch.bfloat16, device=self.flat.device), (Cout, Cin, k)]
            self._cpack_tab = None
        if ent[0] != self.version:
            if self._cpack_next and CONV_PACK_MULTI:
                self._cpack_table()  # a new version: the previous one's forward has used every conv
            if self._cpack_tab is not None and self.flat.is_cuda and CONV_PACK_MULTI:
                tab, nent, mx = self._cpack_tab
                call("es_conv2d_pack_bf16_multi", ptr(tab), nent, mx, _s())
                for e in self._cpack.values():
                    e[0] = self.version
                st = torch.cuda.current_stream(self.flat.device)
                self._cpack_ev = (st, torch.cuda.Event(), {st})
                self._cpack_ev[1].record(st)
            else:
                call("es_conv2d_pack_bf16", ptr(self.pview(name)), Cout, Cin, k, k, ptr(ent[1]), ptr(ent[2]), _s())
                ent[0] = self.version
                self._cpack_next = True  # build the table once this version's weights are all seen
        elif self._cpack_ev is not None:
            st = torch.cuda.current_stream(self.flat.device)
            if st not in self._cpack_ev[2]:  # once per stream and version
                st.wait_event(self._cpack_ev[1])
                self._cpack_ev[2].add(st)
        return ent[1], ent[2]

    def _cpack_table(self):
        """The device table of every conv weight seen so far (es_conv2d_pack_bf16_multi)."""
        self._cpack_next = False
        if not self.flat.is_cuda or not self._cpack:
            return
        esz = _lib.load().es_conv_pack_entry_size()
        ents = list(self._cpack.items())
        raw = bytearray(esz * len(ents))
        mx = 0
        for j, (name, (_, wp, wt, (Cout, Cin, k))) in enumerate(ents):
            entry = (ctypes.c_void_p(ptr(self.pview(name))), ctypes.c_void_p(ptr(wp)), ctypes.c_void_p(ptr(wt)),
                     ctypes.c_int(Cout), ctypes.c_int(Cin), ctypes.c_int(k * k), ctypes.c_int(0))
            buf = b"".join(bytes(e) for e in entry)
            raw[j * esz:j * esz + len(buf)] = buf
            mx = max(mx, Cout * Cin * k * k)
        self._cpack_tab = (torch.frombuffer(raw, dtype=torch.uint8).to(self.flat.device), len(ents), mx)

    def bwd_scratch(self, name, shape, dtype):
        """Zero-initialised scratch for the transformer blocks' backward, allocated once per shape."""
        if not hasattr(self, "_bwd_scratch"):
            self._bwd_scratch = {}
        key = (name, tuple(shape), dtype, self.flat.device)
        t = self._bwd_scratch.get(key)
        if t is None:
            t = self._bwd_scratch[key] = torch.zeros(*shape, dtype=dtype, device=self.flat.device)
        return t

    # ---- parameters: views of one flat buffer; BN running stats: module buffers ------------
    def _resolve(self, name):
        parts = name.split(".")
        mod = self
        for p in parts[:-1]:
            if p not in mod._modules:
                mod._modules[p] = nn.Module()
            mod = mod._modules[p]
        return mod, parts[-1]

    def _build(self, flat, device, buffers=None):
        self.flat = flat
        self.flat_grad = torch.zeros_like(flat)
        for name, shape, kind in self.layout:
            mod, attr = self._resolve(name)
            if kind == "p":
                view = flat[self.offs[name]:self.offs[name] + math.prod(shape)].view(shape)
                mod._parameters[attr] = nn.Parameter(view, requires_grad=True)
            else:
                if buffers is not None:
                    t = buffers[name]
                elif kind == "rm":
                    t = torch.zeros(shape, device=device)
                elif kind == "rv":
                    t = torch.ones(shape, device=device)
                else:
                    t = torch.zeros((), dtype=torch.int64, device=device)
                mod._buffers[attr] = t
        self._packed_version = -1
        self._wtab = None
        self._cpack = {}
        self._cpack_tab, self._cpack_ev, self._cpack_next = None, None, False
        self._bn_partials = {}
        self._anchor = torch.zeros((), device=device, requires_grad=True)

    def _apply(self, fn, recurse=True):
        new = fn(self.flat)
        bufs = {name: fn(self.get_buffer(name)) for name, _, kind in self.layout if kind != "p"}
        self._build(new.contiguous(), device=new.device, buffers=bufs)
        return self

    def __deepcopy__(self, memo):
        other = type(self).__new__(type(self))
        nn.Module.__init__(other)
        other.cfg, other.layout, other.offs, other.numel, other.shapes = (self.cfg, self.layout, self.offs,
                                                                          self.numel, self.shapes)
        bufs = {name: self.get_buffer(name).detach().clone() for name, _, kind in self.layout if kind != "p"}
        other._build(self.flat.detach().clone(), device=self.flat.device, buffers=bufs)
        other.version, other.cur_n = 0, 0
        other.conv_bf16 = self.conv_bf16
        other.train(self.training)
        return other

    def mark_updated(self):
        self.version += 1

    def load_state_dict(self, state_dict, strict=True):
        r = super().load_state_dict(state_dict, strict=strict)
        self.mark_updated()
        return r

    def pview(self, name):
        return self.flat[self.offs[name]:self.offs[name] + math.prod(self.shapes[name])]

    def gview(self, name):
        return self.flat_grad[self.offs[name]:self.offs[name] + math.prod(self.shapes[name])]

    def bn_buffers(self, pre):
        return (self.get_buffer(pre + "running_mean"), self.get_buffer(pre + "running_var"),
                self.get_buffer(pre + "num_batches_tracked"))

    @property
    def fc(self):  # SemiFormer freezes conv_cls_head / trans_cls_head; FixMatch-style callers ask for .fc
        return self.trans_cls_head

    def no_weight_decay(self):
        """Conformer.no_weight_decay (code/models/conformer.py:414-415)."""
        return {"cls_token"}

    def _pack(self):
        """bf16 images W [N, K] / W^T [K, N] of every transformer-block matrix (re-packed after
        each optimizer step, es_pack_weights)."""
        if self._wtab is None:
            D, Hd = self.cfg.dim, self.cfg.hidden
            pres = ["trans_1."] + [s[0] + ".trans_block." for s in self.cfg.stages()]
            mats = []
            for pre in pres:
                mats += [(pre + "attn.qkv.weight", 3 * D, D), (pre + "attn.proj.weight", D, D),
                         (pre + "mlp.fc1.weight", Hd, D), (pre + "mlp.fc2.weight", D, Hd)]
            dev = self.flat.device
            self.wb, self.wt = {}, {}
            esz = _lib.load().es_pack_entry_size()
            raw = bytearray(esz * len(mats))
            for j, (name, N, K) in enumerate(mats):
                self.wb[name] = torch.zeros(N, K, dtype=torch.bfloat16, device=dev)
                self.wt[name] = torch.zeros(K, N, dtype=torch.bfloat16, device=dev)
                entry = (ctypes.c_long(self.offs[name]), ctypes.c_void_p(self.wb[name].data_ptr()),
                         ctypes.c_void_p(self.wt[name].data_ptr()), ctypes.c_int(N), ctypes.c_int(K))
                buf = b"".join(bytes(e) for e in entry)
                raw[j * esz:j * esz + len(buf)] = buf
            self._wtab = (torch.frombuffer(raw, dtype=torch.uint8).to(dev), len(mats))
        if self._packed_version != self.version:
            tab, nmat = self._wtab
            call("es_pack_weights", ptr(self.flat), ptr(tab), nmat, _lib.stream())
            self._packed_version = self.version

    # ---- forward (code/models/conformer.py:418-445) ------------------------------------------
    def _conv_block(self, pre, x, stride, res_conv, x_t=None, return_x2=True):
        """ConvBlock.forward (:107-144).  Without return_x2, x2 feeds conv3 alone: bn2 + ReLU are applied by
        conv3's gathers (bn_conv)."""
        sink = _GradSink() if GRAD_SINKS else None
        x2 = self._conv_block_head(pre, x, stride, x_t, sink=sink, raw_x2=not return_x2)
        out = self._conv_block_tail(pre, x, x2, stride, res_conv, sink=sink, x2_raw=not return_x2)
        return (out, x2) if return_x2 else out

    def _conv_block_head(self, pre, x, stride, x_t=None, sink=None, raw_x2=False):
        """conv1 -> bn1 -> ReLU (-> + upsampled x_t) -> conv2 -> bn2 -> ReLU: x2 (:118-130).  sink: the
        _GradSink x shares with the tail's residual.  Without the FCUUp add, bn1 + ReLU are applied by conv2's
        gathers (bn_conv); raw_x2: return conv2's output before bn2 (the tail's conv3 applies it)."""
        med = self.shapes[pre + "conv1.weight"][0]
        h = conv(self, x, _Map.nhwc(x), pre + "conv1.weight", None, med, 1, stats=True, sink=sink)
        if x_t is not None:
            h = _UpsampleAddFn.apply(bn(self, h, pre + "bn1.", relu=True), x_t, h.shape[1] // x_t.shape[1])
            h = conv(self, h, _Map.nhwc(h), pre + "conv2.weight", None, med, 3, stride, 1, stats=True)
        else:
            h = bn_conv(self, h, pre + "bn1.", pre + "conv2.weight", None, med, 3, stride, 1, stats=True)
        return h if raw_x2 else bn(self, h, pre + "bn2.", relu=True)

    def _conv_block_tail(self, pre, x, x2, stride, res_conv, sink=None, x2_raw=False):
        """conv3 -> bn3 (+ residual, via residual_conv / residual_bn) -> ReLU (:132-144).  x2_raw: x2 is conv2's
        output before bn2 + ReLU, which conv3 applies (bn_conv)."""
        outp = self.shapes[pre + "conv3.weight"][0]
        if x2_raw:
            h = bn_conv(self, x2, pre + "bn2.", pre + "conv3.weight", None, outp, 1, stats=True)
        else:
            h = conv(self, x2, _Map.nhwc(x2), pre + "conv3.weight", None, outp, 1, stats=True)
        residual = x
        if res_conv:
            r = conv(self, x, _Map.nhwc(x), pre + "residual_conv.weight", None, outp, 1, stride, stats=True,
                     sink=sink)
            residual = bn(self, r, pre + "residual_bn.")
            return bn(self, h, pre + "bn3.", relu=True, res=residual)
        return bn(self, h, pre + "bn3.", relu=True, res=residual, res_sink=sink)

    def forward(self, x):
        cfg = self.cfg
        if not self.flat.is_cuda:
            raise _lib.EndosslCallError("NativeConformer runs on the MI355X only: move it to a cuda device first")
        if x.dim() != 4 or x.shape[1:] != (3, cfg.img_size, cfg.img_size):
            raise ValueError(f"expected [n, 3, {cfg.img_size}, {cfg.img_size}] images, got {tuple(x.shape)}")
        if x.dtype == torch.uint8:
            # raw pixels (the host input path's batches): ToTensor + Normalize (code/dataset.py:21-22,49-51)
            # on the device, the same fp32 operations in the same order as torchvision's on the host
            # (divisors as device tensors: torch divides by a Python scalar as a multiply by its
            # reciprocal on the GPU, which is not the host's x / 255 to the last bit)
            mean = torch.tensor(IMAGENET_MEAN, device=x.device).view(1, 3, 1, 1)
            std = torch.tensor(IMAGENET_STD, device=x.device).view(1, 3, 1, 1)
            x = x.float().div_(torch.tensor(255.0, device=x.device)).sub_(mean).div_(std)
        self._pack()
        # a backward that raised after queueing its stream join never ran the callback that clears
        # its key: every new graph starts with no join pending
        _join_queued.clear()
        self._bn_partials.clear()
        x = x.float().contiguous()
        n, S = x.shape[0], cfg.img_size
        self.cur_n = n
        D = cfg.dim
        # stem: conv1 7x7/2 -> bn1 -> ReLU -> maxpool 3/2.  The NCHW images are re-laid NHWC once (a
        # layout copy): the implicit-GEMM gathers then read the 3 channels of a tap from one 12-byte
        # run instead of three planes S^2 apart (stem forward / weight gradient 2-3x faster)
        x = x.permute(0, 2, 3, 1).contiguous()
        img = _Map(x, n, S, S, 3, sn=3 * S * S, sh=3 * S, sw=3, sc=1)
        # the parameters are not autograd inputs (their gradients go straight to flat_grad): a leaf that
        # requires grad, passed to the stem conv, puts the graph on the tape in training mode.  With a
        # frozen trunk (IS_FREEZE) the leaf goes to the two heads instead: only they run a backward
        on_tape = torch.is_grad_enabled() and self.training
        frozen = getattr(self, "frozen_trunk", False)
        anchor = self._anchor if (on_tape and not frozen) else None
        h = conv(self, x, img, "conv1.weight", None, 64, 7, 2, 3, anchor=anchor, out_dtype=torch.float32)
        x_base = _MaxPoolFn.apply(bn(self, h, "bn1.", eps=BN_EPS_STEM, relu=True), 3, 2, 1, _map_dtype(self))
        main = torch.cuda.current_stream(x.device)
        tb = _branch_stream(x.device) if BRANCH_STREAMS else main

        def to_branch(t):  # main-stream tensor read by the branch stream
            if tb is not main:
                tb.wait_stream(main)
                t.record_stream(tb)

        def to_main(t):  # branch-stream tensor read by the main stream
            if tb is not main:
                main.wait_stream(tb)
                t.record_stream(main)

        to_branch(x_base)
        with torch.cuda.stream(tb):
            xt = _PatchTokensFn.apply(x_base, self)
            xt = _BlockFn.apply(xt, self, "trans_1.")
        xc = self._conv_block("conv_1.", x_base, 1, True, return_x2=False)
        T, g = cfg.T, cfg.grid
        stages = list(cfg.stages())
        tsink = None  # the token buffer's gradient sink between a block's FCUUp and the next block's FCUDown
        for si, (name, _, outp, res_conv, stride, dw, last) in enumerate(stages):
            pre = name + "."
            med = outp // 4
            xin = xc
            sink = _GradSink() if GRAD_SINKS else None
            x2 = self._conv_block_head(pre + "cnn_block.", xin, stride, sink=sink)
            to_branch(x2)
            with torch.cuda.stream(tb):
                xt, up, tsink = self._trans_branch(pre, x2, xt, dw, med, tsink, si == len(stages) - 1)
            xc = self._conv_block_tail(pre + "cnn_block.", xin, x2, stride, res_conv, sink=sink)
            to_main(up)
            xc = self._conv_block(pre + "fusion_block.", xc, 2 if last else 1, last, x_t=up, return_x2=False)
        to_main(xt)
        head_anchor = self._anchor if (on_tape and frozen) else None
        conv_cls = _ConvHeadFn.apply(xc, self, head_anchor)
        trans_cls = _TransHeadFn.apply(xt, self, head_anchor)
        return conv_cls, trans_cls

    def _trans_branch(self, pre, x2, xt, dw, med, sink_in=None, final=False):
        """FCUDown -> transformer block -> FCUUp of one ConvTransBlock (:334-352); returns the new token
        buffer, the FCUUp map the fusion block adds and the gradient sink of the new token buffer.  That
        buffer feeds this block's FCUUp conv and the next block's FCUDown (`x_st + x_t`): with GRAD_SINKS
        the two backward contributions are summed in place (_GradSink; in either order -- the FCUDown
        backward has an accumulate form) instead of by autograd's add over [n*T, D] fp32 (S1: 12 adds of
        ~100-146 us); the final block's buffer also feeds the transformer head, so it keeps autograd's add."""
        cfg, n = self.cfg, self.cur_n
        D, T, g = cfg.dim, cfg.T, cfg.grid
        # FCUDown (:161-170): 1x1 conv (bias) -> avg-pool dw -> LN -> GELU -> cat(cls), + x_t.
        # The 1x1 conv and the average pool are both linear maps over different axes (channels /
        # pixels; the pool averages bias-shifted values to the same bias), so they commute: pooling
        # the med-channel map first runs the D-channel conv at 1/dw^2 of the pixels (exact in real
        # arithmetic; fp32 rounding order only)
        x2p = _AvgPoolFn.apply(x2, dw) if dw > 1 else x2
        pooled = conv(self, x2p, _Map.nhwc(x2p), pre + "squeeze_block.conv_project.weight",
                      pre + "squeeze_block.conv_project.bias", D, 1, out_dtype=torch.float32)
        xt = _FcuTokensFn.apply(pooled, xt, self, pre + "squeeze_block.", sink_in)
        xt = _BlockFn.apply(xt, self, pre + "trans_block.")
        # FCUUp (:187-194): token rows 1.. as a [n, g, g, D] map -> 1x1 conv (bias) -> BN -> ReLU;
        # the nearest upsampling is fused into the fusion block's conv2 input
        tok = _Map(xt, n, g, g, D, sn=T * D, sh=g * D, sw=D, sc=1, off=D)
        sink_out = _GradSink() if (GRAD_SINKS and TOKEN_SINK and not final) else None
        up = conv(self, xt, tok, pre + "expand_block.conv_project.weight", pre + "expand_block.conv_project.bias",
                  med, 1, stats=True, sink=sink_out)
        up = bn(self, up, pre + "expand_block.bn.", relu=True)
        return xt, up, sink_out
