"""CPU checks of the ResNet-18 plumbing (no GPU): the native model's state_dict is timm resnet18's
layout (names, order, shapes, 11,188,311 parameters at 23 classes), build_model selects it, and the
oracle's restatement runs a train-mode step on that state (finite loss, every parameter gets a
gradient, BatchNorm buffers advance)."""
import torch

from oracle import resnet_ref as rr
from oracle.conformer_ref import is_buffer


def test_resnet18_layout_and_oracle_step():
    from endossl.build import build_model
    from endossl.resnet import NativeResNet
    from endossl.utils import AttrDict
    m = build_model(AttrDict(MODEL=AttrDict(NAME="resnet18", NUM_CLASSES=23, PRE_TRAIN_PATH="None"),
                             DATA=AttrDict(IMG_SIZE=224)))
    assert isinstance(m, NativeResNet)
    sd = m.state_dict()
    names = list(sd)
    assert names[:2] == ["conv1.weight", "bn1.weight"] and names[-2:] == ["fc.weight", "fc.bias"]
    assert "layer2.0.downsample.0.weight" in sd and "layer1.0.downsample.0.weight" not in sd
    assert sum(v.numel() for k, v in sd.items() if not is_buffer(k)) == 11_188_311
    assert sd["layer4.1.conv2.weight"].shape == (512, 512, 3, 3) and sd["fc.weight"].shape == (23, 512)
    g = torch.Generator().manual_seed(0)
    x, y = torch.randn(4, 3, 64, 64, generator=g), torch.randint(0, 23, (4,), generator=g)
    r = rr.SupervisedRef(sd, class_weights=torch.linspace(0.5, 2.0, 23))
    out = r.step(x, y)
    assert torch.isfinite(torch.tensor(out["loss"]))
    assert all(torch.isfinite(v).all() and v.abs().sum() > 0 for k, v in out["grads"].items())
    assert int(r.bufs["bn1.num_batches_tracked"]) == 1
