"""The host input path feeding the device step: HostBatcher's pinned uint8
batches reach the GPU unchanged, the device's fused ToTensor + Normalize over them equals the
reference's host normalisation (code/dataset.py:49-51) of the same pixels, and a FixMatch step runs
on them."""
import numpy as np
import pytest
import torch

from endossl import host_aug
from endossl._lib import call, ptr

pytestmark = pytest.mark.gpu

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def _sources(n, seed=0):
    g = np.random.default_rng(seed)
    base = g.integers(0, 256, (40, 52, 3), dtype=np.uint8)
    return [host_aug.resize_bilinear(base ^ np.uint8(i * 37 % 256), (300 + 7 * i, 220 + 5 * i)) for i in range(n)]


def test_batcher_device_batches_equal_host_transform():
    srcs = _sources(6)
    hb = host_aug.HostBatcher(srcs, batch=8, size=64, seed=3, threads=4, device="cuda")
    for step in range(3):
        w, s = hb.next()
        idx = hb._indices(step)
        rw, rs = host_aug.transform_batch([srcs[i] for i in idx], 64, "fixmatch", True, seed=(3 << 32) ^ step,
                                          threads=1)
        torch.cuda.synchronize()
        assert w.is_cuda and s.is_cuda
        assert torch.equal(w.cpu(), rw) and torch.equal(s.cpu(), rs)


def test_device_normalisation_of_host_batches_matches_reference():
    """es_patch_im2col_u8 over a host-augmented batch == es_patch_im2col over ToTensor + Normalize of the
    same uint8 pixels done on the host in fp32 (bit-identical bf16 patches)."""
    srcs = _sources(4)
    w, s = host_aug.transform_batch(srcs, 224, "fixmatch", True, seed=9, threads=4)
    u8 = s.cuda()
    n, S, P = u8.shape[0], 224, 16
    mean = torch.tensor(MEAN).view(1, 3, 1, 1)
    std = torch.tensor(STD).view(1, 3, 1, 1)
    f32 = ((s.float() / 255.0 - mean) / std).cuda()
    rows = n * (S // P) ** 2
    pa = torch.zeros(rows, 3 * P * P, dtype=torch.bfloat16, device="cuda")
    pb = torch.zeros_like(pa)
    from endossl import _lib
    stream = _lib.stream()
    call("es_patch_im2col_u8", ptr(u8), *MEAN, *STD, ptr(pa), n, S, P, stream)
    call("es_patch_im2col", ptr(f32), ptr(pb), n, S, P, stream)
    torch.cuda.synchronize()
    assert torch.equal(pa, pb)


def test_fixmatch_step_on_host_batches():
    from endossl.fixmatch import FixMatch
    from endossl.utils import AttrDict
    from endossl.vit import NativeViT, ViTConfig
    B, MU = 2, 2
    model = NativeViT(ViTConfig(depth=2), seed=0)
    tr = FixMatch(model, device=torch.device("cuda"))
    cfg = AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=224, TARGET_NAME="target"),
                   MODEL=AttrDict(NAME="vit_small_patch16_224", NUM_CLASSES=23),
                   TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                  CLS_WEIGHT=False, THRES=0.5, T=1.0, LAMBDA_U=1.0, EPOCHS=1, WARMUP_EPOCHS=0,
                                  DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const"))
    tr.get_dataloader((None, None), None)
    tr.get_config(cfg)
    srcs = _sources(5)
    lab = host_aug.HostBatcher(srcs, batch=B, size=224, kind="labeled", seed=1, threads=2)
    unl = host_aug.HostBatcher(srcs, batch=B * MU, size=224, kind="fixmatch", seed=2, threads=2)
    for _ in range(2):
        (x,) = lab.next()
        uw, us = unl.next()
        y = torch.randint(0, 23, (B,), device="cuda")
        out = tr.step(((x, y), ((uw, us), None)))
    torch.cuda.synchronize()
    assert torch.isfinite(out["loss"]).item()


def test_conformer_uint8_input_equals_host_normalised():
    """NativeConformer fed raw uint8 pixels (the host input path's batches) normalises them on the
    device with torchvision's fp32 operations: the same logits as the host-normalised fp32 images."""
    from endossl.conformer import ConformerConfig, NativeConformer
    kw = dict(img_size=64, patch=16, base_channel=64, channel_ratio=1, embed_dim=128, depth=3, heads=2, num_classes=23)
    m = NativeConformer(ConformerConfig(**kw), seed=3).to("cuda")
    m.eval()
    srcs = _sources(3)
    (x8,) = host_aug.transform_batch(srcs, 64, "eval", True, threads=2)
    mean = torch.tensor(MEAN).view(1, 3, 1, 1)
    std = torch.tensor(STD).view(1, 3, 1, 1)
    xf = (x8.float() / 255.0 - mean) / std  # ToTensor + Normalize on the host (code/dataset.py:49-51)
    with torch.no_grad():
        a = [t.clone() for t in m(x8.cuda())]
        b = [t.clone() for t in m(xf.cuda())]
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
