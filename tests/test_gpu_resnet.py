"""ResNet-18 + the supervised trainer on the MI355X (BASELINE configs[0], code/supervised.py).

The native ResNet-18 (endossl/resnet.py, the Conformer's conv / BatchNorm / pooling kernels) against
the oracle's restatement of timm's resnet18 (oracle/resnet_ref.py; parity against timm itself is
unpinned -- timm is absent and no reference fixture holds a ResNet output): with fp32 convs the
logits within 1e-3 of scale and every gradient within 2e-3 |g| + 4x the fp32 oracle's own distance from
fp64 (BatchNorm-amplified summation order); with the default bf16 convs the
device within twice the bf16-contract emulation's distance from fp32 (the criterion of
test_gpu_conformer.py: BatchNorm passes the rounding flips of the device's own conv inputs on); the
emulation rounds the maps where the device stores them bf16 (NativeResNet.map_bf16).
SupLearning.step against the oracle's step: loss, EMA and BatchNorm buffers, parameters after Adam.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import resnet_ref as rr  # noqa: E402
from oracle.conformer_ref import is_buffer  # noqa: E402

DEV = "cuda"


def _model(seed=2, conv="fp32"):
    from endossl.resnet import NativeResNet, ResNetConfig
    m = NativeResNet(ResNetConfig(num_classes=23), seed=seed)
    state = {k: v.detach().clone() for k, v in m.state_dict().items()}
    return m.to(DEV).set_conv_precision(conv), state


@pytest.mark.parametrize("conv", ["fp32", "bf16"])
def test_resnet18_forward_backward_vs_oracle(conv):
    m, state = _model(conv=conv)
    x = torch.randn(8, 3, 64, 64, generator=torch.Generator().manual_seed(3))
    res = {}
    for bf in (True, False, "f64"):
        dt = torch.float64 if bf == "f64" else torch.float32
        p = {k: v.clone().to(dt).requires_grad_(True) for k, v in state.items() if not is_buffer(k)}
        bufs = {k: (v.clone().to(dt) if v.is_floating_point() else v.clone()) for k, v in state.items()
                if is_buffer(k)}
        out = rr.resnet18_forward(p, bufs, x.to(dt), train=True, bf16=bf is True and conv == "bf16", maps=m.map_bf16)
        res[bf] = (out, p, bufs)
    m.train()
    m.flat_grad.zero_()
    h = m(x.to(DEV))
    r16, r32 = res[True][0].detach().double(), res[False][0].detach().double()
    sc = max(1.0, r32.abs().max().item())
    hd = h.detach().cpu().double()
    e16, e32, env = (hd - r16).abs().max().item(), (hd - r32).abs().max().item(), (r16 - r32).abs().max().item()
    if conv == "bf16":
        assert e32 <= 2 * env + 1e-3 * sc, (e32, env, sc)
    else:
        assert e32 <= 1e-3 * sc, (e32, sc)
    for k in ("bn1.running_mean", "layer3.0.downsample.1.running_var", "layer4.1.bn2.running_mean"):
        ref = res[True][2][k]
        assert (m.get_buffer(k).cpu() - ref).abs().max().item() <= (2e-2 if conv == "bf16" else 1e-3) * max(
            1.0, ref.abs().max().item()), k
    g = torch.randn(h.shape, generator=torch.Generator().manual_seed(4))
    (h * g.to(DEV)).sum().backward()
    grads = {}
    for bf in (True, False, "f64"):
        out, p, _ = res[bf]
        (out * g.to(out.dtype)).sum().backward()
        grads[bf] = {k: v.grad for k, v in p.items()}
    gmax = max(grads[False][k].double().norm().item() for k in grads[False])
    bad = []
    for k in grads[False]:
        gh = m.gview(k).cpu().view(grads[False][k].shape).double()
        g16, g32 = grads[True][k].double(), grads[False][k].double()
        nrm = g32.norm().item()
        if conv == "bf16":
            e, env = (gh - g32).norm().item(), 2 * (g16 - g32).norm().item()
        else:
            # fp32 convs: the device against fp64, within 4x the fp32 oracle's own distance from fp64 --
            # 18 BatchNorm layers over 8 images at 64^2 (32 values per channel in layer4) amplify fp32
            # summation-order noise to a few 1e-3 of |g| in the deep layers' and the stem's gradients
            g64 = grads["f64"][k].double()
            e, env = (gh - g64).norm().item(), 4 * (g32 - g64).norm().item()
        if e > 2e-3 * nrm + env + 1e-4 * gmax:
            bad.append((k, e, env, nrm))
    assert not bad, bad[:8]


def test_suplearning_step_vs_oracle():
    """Two SupLearning steps (weighted CE, Adam 1e-3, EMA 0.999) against the oracle at the device's own
    pre-step state, fp32 convs: loss to 1e-4 relative; then the trajectory: parameters within 2 lr per
    step of the oracle's (Adam turns a ~0 gradient's sign into +-lr), EMA and BatchNorm buffers."""
    from endossl.supervised import SupLearning
    from endossl.utils import AttrDict
    m, state = _model(seed=5)
    g = torch.Generator().manual_seed(8)
    batches = [(torch.randn(8, 3, 64, 64, generator=g), torch.randint(0, 23, (8,), generator=g)) for _ in range(2)]
    cw = torch.linspace(0.5, 2.0, 23)

    class _DS:
        df = None

    class _DL(list):
        dataset = _DS()

    tr = SupLearning(m, opt_func="Adam", lr=1e-3, device=DEV)
    tr.get_dataloader(_DL(batches), None, None)
    tr.get_config(AttrDict(DATA=AttrDict(BATCH_SIZE=8, IMG_SIZE=64, TARGET_NAME="target"),
                           MODEL=AttrDict(NAME="resnet18", NUM_CLASSES=23, MARGIN="None", IS_TRIPLET=False),
                           TRAIN=AttrDict(USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, CLS_WEIGHT=False, EPOCHS=1,
                                          WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8,
                                          SCH_NAME="const", FREQ_EVAL=1)))
    tr.class_weights = cw.to(DEV)
    traj = rr.SupervisedRef(state, class_weights=cw)
    for i, (x, y) in enumerate(batches):
        snap = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        ref = rr.SupervisedRef(snap, class_weights=cw).step(x, y)
        out = tr.step((x, y))
        traj.step(x, y)
        torch.cuda.synchronize()
        assert abs(out["loss"].item() - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"])), (i, out["loss"], ref["loss"])
    sd, esd = m.state_dict(), tr.ema_model.ema.state_dict()
    for k, v in sd.items():
        if is_buffer(k):
            if k.endswith("num_batches_tracked"):
                assert int(v.item()) == 2 and int(esd[k].item()) == 0  # EMA of an int buffer truncates
            else:
                assert (v.cpu() - traj.bufs[k]).abs().max().item() <= 1e-3 * max(1.0, traj.bufs[k].abs().max().item()), k
            continue
        assert (v.cpu() - traj.p[k].detach()).abs().max().item() <= 2 * 2e-3 + 1e-6, k
        assert (esd[k].cpu() - traj.ema[k]).abs().max().item() <= 1e-3 * 4e-3 + 1e-6, k


def test_suplearning_graph_replay_bit_identical():
    """SupLearning.use_graph: the forward / loss / backward captured once (after GRAPH_WARM eager steps) and
    replayed, new batches copied into the graph's inputs, against every step eager -- losses, logits,
    parameters, EMA and BatchNorm buffers BIT-identical over eight steps (bf16 convs; the captured steps
    pack the conv weights themselves).  The returned tensors are read only after the last step (the graph
    path returns copies, not its static outputs), and a ragged batch between two full ones runs eagerly
    without discarding the captured graph."""
    from endossl.supervised import SupLearning
    from endossl.utils import AttrDict
    g = torch.Generator().manual_seed(11)
    batches = [(torch.randn(8, 3, 64, 64, generator=g), torch.randint(0, 23, (8,), generator=g)) for _ in range(6)]

    class _DS:
        df = None

    class _DL(list):
        dataset = _DS()

    batches.append((torch.randn(5, 3, 64, 64, generator=g), torch.randint(0, 23, (5,), generator=g)))  # ragged last
    batches.append(batches[0])  # the main shape again: its graph survives the ragged batch
    runs = {}
    for graph in (False, True):
        m, _ = _model(seed=6, conv="bf16")
        tr = SupLearning(m, opt_func="Adam", lr=1e-3, device=DEV)
        tr.use_graph = graph
        tr.get_dataloader(_DL(batches), None, None)
        tr.get_config(AttrDict(DATA=AttrDict(BATCH_SIZE=8, IMG_SIZE=64, TARGET_NAME="target"),
                               MODEL=AttrDict(NAME="resnet18", NUM_CLASSES=23, MARGIN="None", IS_TRIPLET=False),
                               TRAIN=AttrDict(USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, CLS_WEIGHT=False,
                                              EPOCHS=1, WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4,
                                              LR_DECAY=0.8, SCH_NAME="const", FREQ_EVAL=1)))
        tr.class_weights = torch.linspace(0.5, 2.0, 23).to(DEV)
        outs = [tr.step((x.to(DEV), y.to(DEV))) for x, y in batches]  # kept un-cloned across later steps
        torch.cuda.synchronize()
        losses = [o["loss"].item() for o in outs]
        logits = [o["logits"].cpu() for o in outs]
        graphs = [e for e in getattr(tr, "_graphs", {}).values() if e["graph"] is not None]
        assert len(graphs) == (1 if graph else 0)
        runs[graph] = (losses, logits, {k: v.detach().cpu().clone() for k, v in m.state_dict().items()},
                       {k: v.detach().cpu().clone() for k, v in tr.ema_model.ema.state_dict().items()})
    (le, ge, se, ee), (lg, gg, sg, eg) = runs[False], runs[True]
    assert le == lg, (le, lg)
    for i, (a, b) in enumerate(zip(ge, gg)):
        assert torch.equal(a, b), i
    for k in se:
        assert torch.equal(se[k], sg[k]), k
        assert torch.equal(ee[k], eg[k]), k
