"""build_model (code/build.py:29-222) for the SSL hot path.

The reference builds its FixMatch backbone with `timm.create_model(name, pretrained=True,
num_classes=C)` (code/build.py:196-197) -- a network weight download, and timm is absent here.
This factory returns the native ViT for the `vit_*` names instead (random timm-style init, or a
checkpoint from MODEL.PRE_TRAIN_PATH loaded with weights_only=True, head dropped when its class
count differs -- the reference re-heads abnormality checkpoints the same way, :180-194).
For MODEL.TYPE_SEMI == 'CoMatch' it returns ModelwEmb over the native ViT (:175-178;
comatch_model.NativeViTEmb, forward -> (logits, fts, z), LOW_DIM-d embedding).
For 'conformer' it returns the native Conformer-Ti of code/build.py:135-142 (patch 16,
channel_ratio 1, embed 384, depth 12, 6 heads, qkv_bias; conformer.NativeConformer, forward ->
(conv_logits, trans_logits)) -- SemiFormer's backbone.  CNN / Swin backbones are outside the
hot path.
"""
import torch

from .comatch_model import NativeViTEmb
from .conformer import ConformerConfig, NativeConformer
from .resnet import NativeResNet, ResNetConfig
from .vit import VIT_CONFIGS, NativeViT, ViTConfig


def build_model(config, is_pathology=True, seed=0):
    name = config.MODEL.NAME
    C = int(config.MODEL.NUM_CLASSES)
    if name == "conformer":
        img = int(config.DATA.IMG_SIZE) if "IMG_SIZE" in config.DATA else 224
        model = NativeConformer(ConformerConfig(img_size=img, patch=16, channel_ratio=1, embed_dim=384, depth=12,
                                                heads=6, mlp_ratio=4, num_classes=C), seed=seed)
        path = getattr(config.MODEL, "PRE_TRAIN_PATH", "None")
        if path not in (None, "None", ""):
            ck = torch.load(path, map_location="cpu", weights_only=True)
            sd = ck.get("model_state_dict", ck)
            sd = {k: v for k, v in sd.items() if not k.startswith(("conv_cls_head.", "trans_cls_head."))
                  or v.shape[0] == C}
            model.load_state_dict(sd, strict=False)
        return model
    if name == "resnet18":
        # the supervised baseline (BASELINE configs[0]; code/build.py:218-220 timm.create_model('resnet18',
        # num_classes=C): ImageNet weights are a download, unavailable here -- timm's random init)
        if getattr(config.MODEL, "PRE_TRAIN_PATH", "None") not in (None, "None", ""):
            raise NotImplementedError("resnet18 + PRE_TRAIN_PATH swaps fc for build_head's MLP "
                                      "(code/build.py:202-211): outside the native scope")
        return NativeResNet(ResNetConfig(num_classes=C), seed=seed)
    if name not in VIT_CONFIGS:
        raise NotImplementedError(f"backbone {name!r}: native builds exist for {sorted(VIT_CONFIGS)}")
    comatch = getattr(config.MODEL, "TYPE_SEMI", "FixMatch") == "CoMatch" and getattr(config.TRAIN, "IS_SSL", True)
    kw = dict(VIT_CONFIGS[name])
    if "IMG_SIZE" in config.DATA and int(config.DATA.IMG_SIZE) != kw["img_size"]:
        kw["img_size"] = int(config.DATA.IMG_SIZE)
    if comatch:
        model = NativeViTEmb(ViTConfig(num_classes=C, head="emb", low_dim=int(config.MODEL.LOW_DIM), **kw), seed=seed)
    else:
        model = NativeViT(ViTConfig(num_classes=C, **kw), seed=seed)
    path = getattr(config.MODEL, "PRE_TRAIN_PATH", "None")
    if path not in (None, "None", ""):
        ck = torch.load(path, map_location="cpu", weights_only=True)
        sd = ck.get("model_state_dict", ck)
        if sd.get("head.weight") is not None and sd["head.weight"].shape[0] != C:
            sd = {k: v for k, v in sd.items() if not k.startswith("head.")}
        model.load_state_dict(sd, strict=False)
    return model
