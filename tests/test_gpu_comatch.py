"""CoMatch on the MI355X: every CoMatch C-ABI kernel against a plain torch fp32 restatement of the
reference arithmetic (autograd for the gradients), and the native CoMatch trainer against the
reference's own CoMatch.train_one fixtures (tests/golden/comatch_step_{open,closed}.npz, bank
gate open / closed), replaying the reference's dropout masks.

Bars: kernels within fp32 tolerances (rtol 1e-4 .. 1e-5).  Trainer, step 0: trunk features within
1e-3 * scale (+ a quarter of the bf16 envelope) of the bf16-contract oracle; every later stage
(heads, DA / smoothing, losses, dL/dlogits, dL/dz, heads backward) within fp32 tolerances of the
oracle run on the HIP path's own stage inputs; pseudo-labels / masks bit-exact on decidable rows.
Trajectory (both steps): |HIP - reference| <= 1.5 * |bf16 contract - reference| + tol for logits,
losses, DA history, bank, BN buffers; post-step params within 2 * lr * steps (+1e-5).
"""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from endossl import _lib  # noqa: E402
from endossl._lib import call, ptr  # noqa: E402
from oracle import ref  # noqa: E402

DEV = "cuda"


def S():
    return _lib.stream()


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    _lib.load()


# ------------------------------------------------------------------------------------- kernels
@pytest.mark.parametrize("n,T,D", [(5, 17, 128), (9, 197, 384)])
def test_cls_ln_fwd_bwd(n, T, D):
    torch.manual_seed(n)
    x = torch.randn(n * T, D, device=DEV) * 2 + 0.3
    g = 1 + 0.1 * torch.randn(D, device=DEV)
    b = 0.1 * torch.randn(D, device=DEV)
    fts = torch.zeros(n, D, device=DEV)
    xhat, rstd = torch.zeros(n, D, device=DEV), torch.zeros(n, device=DEV)
    call("es_cls_ln_fwd", ptr(x), D, T, ptr(g), ptr(b), ptr(fts), D, ptr(xhat), ptr(rstd), n, D, 1e-6, S())
    xr = x.view(n, T, D)[:, 0].clone().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.layer_norm(xr, (D,), gr, br, 1e-6)
    torch.testing.assert_close(fts, yr.detach(), rtol=1e-5, atol=1e-5)
    dy = torch.randn(n, D, device=DEV)
    yr.backward(dy)
    dx = torch.full((n * T, D), 7.0, device=DEV)
    dg, db = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    call("es_cls_ln_bwd", ptr(dy), D, ptr(g), ptr(xhat), ptr(rstd), ptr(dx), D, T, ptr(dg), ptr(db), n, D, S())
    torch.testing.assert_close(dx.view(n, T, D)[:, 0], xr.grad, rtol=1e-4, atol=1e-4)
    assert torch.all(dx.view(n, T, D)[:, 1:] == 7.0)  # only CLS rows written
    torch.testing.assert_close(dg, gr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("with_keep", [False, True])
@pytest.mark.parametrize("N", [96, 23])  # 23: the few-column forward (one wave per output)
def test_dense_fwd_bwd(act, with_keep, N):
    torch.manual_seed(act * 2 + with_keep + N)
    n, K = 37, 384
    X = torch.randn(n, K, device=DEV)
    W = torch.randn(N, K, device=DEV) * 0.05
    b = torch.randn(N, device=DEV) * 0.1
    keep = (torch.rand(n, N, device=DEV) >= 0.2).to(torch.uint8) if with_keep else None
    scale = 1.25
    Y = torch.zeros(n, N, device=DEV)
    call("es_dense_fwd", ptr(X), K, ptr(W), ptr(b), ptr(Y), N, n, K, N, act, 0.1, ptr(keep) if with_keep else None,
         scale, S())
    Xr, Wr, br = (t.clone().requires_grad_(True) for t in (X, W, b))
    pre = Xr @ Wr.t() + br
    y = pre if act == 0 else (F.relu(pre) if act == 1 else F.leaky_relu(pre, 0.1))
    if with_keep:
        y = y * keep.float() * scale
    torch.testing.assert_close(Y, y.detach(), rtol=1e-5, atol=1e-5)
    dY = torch.randn(n, N, device=DEV)
    y.backward(dY)
    dX = torch.full((n, K), 0.5, device=DEV)
    dW, db = torch.zeros(N, K, device=DEV), torch.zeros(N, device=DEV)
    ws = torch.zeros(_lib.load().es_dense_bwd_workspace(n, N), device=DEV)
    call("es_dense_bwd", ptr(dY), N, ptr(Y) if act else None, N, act, 0.1, ptr(keep) if with_keep else None, scale,
         ptr(X), K, ptr(W), ptr(dX), K, 1, ptr(dW), ptr(db), n, K, N, ptr(ws), S())
    torch.testing.assert_close(dX, Xr.grad + 0.5, rtol=1e-4, atol=1e-4)  # accumulate = 1
    torch.testing.assert_close(dW, Wr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("n,Fe", [(1408, 96), (14, 32), (2, 8)])
def test_bn1d_fwd_bwd(n, Fe):
    torch.manual_seed(n)
    U = torch.randn(n, Fe, device=DEV) * 1.7 + 0.4
    g = 1 + 0.1 * torch.randn(Fe, device=DEV)
    bt = 0.1 * torch.randn(Fe, device=DEV)
    rm, rv = torch.randn(Fe, device=DEV) * 0.1, 1 + torch.rand(Fe, device=DEV)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    rm_ref, rv_ref = rm.clone(), rv.clone()
    Y, xhat, rstd = torch.zeros(n, Fe, device=DEV), torch.zeros(n, Fe, device=DEV), torch.zeros(Fe, device=DEV)
    call("es_bn1d_fwd", ptr(U), Fe, ptr(g), ptr(bt), ptr(rm), ptr(rv), ptr(nbt), 0.1, 1e-5, 1, ptr(Y), Fe, ptr(xhat),
         ptr(rstd), n, Fe, S())
    Ur, gr, br = (t.clone().requires_grad_(True) for t in (U, g, bt))
    y = F.batch_norm(Ur, rm_ref, rv_ref, gr, br, training=True, momentum=0.1, eps=1e-5)
    torch.testing.assert_close(Y, y.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rm, rm_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv, rv_ref, rtol=1e-5, atol=1e-6)
    assert int(nbt.item()) == 1
    dY = torch.randn(n, Fe, device=DEV)
    y.backward(dY)
    dU, dg, db = torch.zeros(n, Fe, device=DEV), torch.zeros(Fe, device=DEV), torch.zeros(Fe, device=DEV)
    call("es_bn1d_bwd", ptr(dY), Fe, ptr(xhat), ptr(rstd), ptr(g), ptr(dU), Fe, ptr(dg), ptr(db), n, Fe, S())
    torch.testing.assert_close(dU, Ur.grad, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(dg, gr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-3)
    # eval mode: running statistics
    Y2 = torch.zeros(n, Fe, device=DEV)
    call("es_bn1d_fwd", ptr(U), Fe, ptr(g), ptr(bt), ptr(rm), ptr(rv), None, 0.1, 1e-5, 0, ptr(Y2), Fe, None, None, n,
         Fe, S())
    torch.testing.assert_close(Y2, F.batch_norm(U, rm, rv, g, bt, training=False, eps=1e-5), rtol=1e-5, atol=1e-5)


def test_l2norm_fwd_bwd():
    torch.manual_seed(5)
    n, L = 50, 64
    V = torch.randn(n, L, device=DEV)
    Z, nrm = torch.zeros(n, L, device=DEV), torch.zeros(n, device=DEV)
    call("es_l2norm_fwd", ptr(V), L, ptr(Z), L, ptr(nrm), n, L, S())
    Vr = V.clone().requires_grad_(True)
    z = Vr.div(Vr.pow(2).sum(1, keepdim=True).pow(0.5))  # Normalize(2), code/models/custom_model.py:136-145
    torch.testing.assert_close(Z, z.detach(), rtol=1e-5, atol=1e-6)
    dZ = torch.randn(n, L, device=DEV)
    z.backward(dZ)
    dV = torch.zeros(n, L, device=DEV)
    call("es_l2norm_bwd", ptr(dZ), L, ptr(Z), L, ptr(nrm), ptr(dV), L, n, L, S())
    torch.testing.assert_close(dV, Vr.grad, rtol=1e-4, atol=1e-5)


def _unit(t):
    return t / t.norm(dim=1, keepdim=True)


@pytest.mark.parametrize("Q,zero_bank,nu,L", [(600, False, 448, 64), (2560, True, 448, 64), (65536, False, 448, 64),
                                              (300, False, 37, 40)])
def test_comatch_pseudo_vs_reference_formula(Q, zero_bank, nu, L):
    """DA over a 3-entry history + memory smoothing (code/comatch.py:167-185) vs torch fp64.
    (300, 37, 40): bank, weak-row and embedding sizes off the kernel's 128 / 16 / 4 tiles."""
    torch.manual_seed(Q)
    C, T, alpha, thres = 23, 0.2, 0.9, 0.6
    lw = torch.randn(nu, C, device=DEV) * torch.rand(nu, 1, device=DEV) * 6
    zw = _unit(torch.randn(nu, L, device=DEV))
    bf = torch.zeros(Q, L, device=DEV) if zero_bank else _unit(torch.randn(Q, L, device=DEV))
    bp = torch.zeros(Q, C, device=DEV) if zero_bank else torch.softmax(torch.randn(Q, C, device=DEV) * 3, -1)
    hist = torch.zeros(32, C, device=DEV)
    prev = [torch.softmax(torch.randn(C, device=DEV), -1) for _ in range(2)]
    hist[30], hist[31] = prev  # ring: two older entries at slots 30, 31; the new one goes to slot 0
    probs, porig = torch.zeros(nu, C, device=DEV), torch.zeros(nu, C, device=DEV)
    pl, mask = torch.zeros(nu, dtype=torch.int32, device=DEV), torch.zeros(nu, device=DEV)
    ws = torch.zeros(_lib.load().es_comatch_pseudo_workspace(nu, C, Q), device=DEV)
    call("es_comatch_pseudo", ptr(lw), C, nu, C, ptr(hist), 32, 3, 0, ptr(zw), L, L, ptr(bf), ptr(bp), Q, T, alpha,
         thres, ptr(probs), ptr(porig), ptr(pl), ptr(mask), ptr(ws), S())
    p = torch.softmax(lw.double(), 1)
    plist = [t.double() for t in prev] + [p.mean(0)]
    torch.testing.assert_close(hist[0].double(), plist[-1], rtol=1e-5, atol=1e-7)
    p = p / torch.stack(plist).mean(0)
    p = p / p.sum(1, keepdim=True)
    torch.testing.assert_close(porig.double(), p, rtol=1e-5, atol=1e-7)
    A = torch.exp(zw.double() @ bf.double().t() / T)
    A = A / A.sum(1, keepdim=True)
    p = alpha * p + (1 - alpha) * A @ bp.double()
    torch.testing.assert_close(probs.double(), p, rtol=1e-5, atol=1e-6)
    sc, lb = p.max(1)
    top2 = p.topk(2, 1).values
    ok = (top2[:, 0] - top2[:, 1]) > 1e-5
    assert torch.equal(pl.long()[ok], lb[ok])
    okm = (sc - thres).abs() > 1e-5
    assert torch.equal(mask.bool()[okm], (sc >= thres)[okm])


def test_softmax_colmean_and_given_history():
    """The data-parallel DA path: es_softmax_colmean = mean softmax, and es_comatch_pseudo_ex with
    hist_given = 1 uses the caller's hist[pos] instead of the local batch mean."""
    torch.manual_seed(17)
    nu, C, L, Q = 96, 23, 64, 640
    lw = torch.randn(nu, C, device=DEV) * 4
    out = torch.empty(C, device=DEV)
    call("es_softmax_colmean", ptr(lw), C, nu, C, ptr(out), S())
    torch.testing.assert_close(out, torch.softmax(lw.double(), 1).mean(0).float(), rtol=1e-5, atol=1e-7)
    zw = _unit(torch.randn(nu, L, device=DEV))
    bf, bp = _unit(torch.randn(Q, L, device=DEV)), torch.softmax(torch.randn(Q, C, device=DEV), -1)
    ws = torch.zeros(_lib.load().es_comatch_pseudo_workspace(nu, C, Q), device=DEV)
    given = torch.softmax(torch.randn(C, device=DEV), -1)  # e.g. the all-ranks mean
    res = []
    for flag in (0, 1):
        hist = torch.zeros(32, C, device=DEV)
        hist[0] = given
        probs, porig = torch.zeros(nu, C, device=DEV), torch.zeros(nu, C, device=DEV)
        pl, mask = torch.zeros(nu, dtype=torch.int32, device=DEV), torch.zeros(nu, device=DEV)
        call("es_comatch_pseudo_ex", ptr(lw), C, nu, C, ptr(hist), 32, 1, 0, flag, ptr(zw), L, L, ptr(bf), ptr(bp), Q,
             0.2, 0.9, 0.5, ptr(probs), ptr(porig), ptr(pl), ptr(mask), ptr(ws), S())
        res.append((hist[0].clone(), porig.clone()))
    torch.testing.assert_close(res[0][0], out)          # recomputed from the local rows
    torch.testing.assert_close(res[1][0], given)        # kept as given
    p = torch.softmax(lw.double(), 1) / given.double()
    torch.testing.assert_close(res[1][1].double(), p / p.sum(1, keepdim=True), rtol=1e-5, atol=1e-7)


def test_comatch_bank_write():
    torch.manual_seed(2)
    nu, bt, L, C, Q, ptr0 = 14, 2, 16, 23, 48, 16
    zw, zx = torch.randn(nu, L, device=DEV), torch.randn(bt, L, device=DEV)
    po = torch.rand(nu, C, device=DEV)
    y = torch.tensor([3, 22], dtype=torch.int64, device=DEV)
    bf, bp = torch.full((Q, L), 9.0, device=DEV), torch.full((Q, C), 9.0, device=DEV)
    call("es_comatch_bank_write", ptr(zw), L, nu, ptr(zx), L, bt, L, ptr(po), ptr(y), C, ptr(bf), ptr(bp), ptr0, Q, S())
    torch.testing.assert_close(bf[ptr0:ptr0 + nu + bt], torch.cat([zw, zx]), rtol=0, atol=0)
    onehot = torch.zeros(bt, C, device=DEV).scatter(1, y.view(-1, 1), 1)
    torch.testing.assert_close(bp[ptr0:ptr0 + nu + bt], torch.cat([po, onehot]), rtol=0, atol=0)
    assert torch.all(bf[:ptr0] == 9.0) and torch.all(bf[ptr0 + nu + bt:] == 9.0)


@pytest.mark.parametrize("nu", [448, 4])
def test_comatch_contrastive_fwd_bwd(nu):
    torch.manual_seed(nu)
    L, C, T, th, scale = 64, 23, 0.2, 0.8, 2.0 / nu
    z0, z1 = _unit(torch.randn(nu, L, device=DEV)), _unit(torch.randn(nu, L, device=DEV))
    probs = torch.softmax(torch.randn(nu, C, device=DEV) * 4, -1) * 0.9
    loss = torch.zeros(1, device=DEV)
    dz0, dz1 = torch.zeros(nu, L, device=DEV), torch.zeros(nu, L, device=DEV)
    ws = torch.zeros(_lib.load().es_comatch_contrastive_workspace(nu), device=DEV)
    call("es_comatch_contrastive_fwd_bwd", ptr(z0), L, ptr(z1), L, ptr(probs), nu, L, C, T, th, scale, ptr(loss),
         ptr(dz0), L, ptr(dz1), L, ptr(ws), S())
    a, b = z0.clone().requires_grad_(True), z1.clone().requires_grad_(True)
    sim = torch.exp(a @ b.t() / T)  # code/comatch.py:200-213
    sp = sim / sim.sum(1, keepdim=True)
    Qm = probs @ probs.t()
    Qm.fill_diagonal_(1)
    Qm = Qm * (Qm >= th).float()
    Qm = Qm / Qm.sum(1, keepdim=True)
    lc = -(torch.log(sp + 1e-7) * Qm).sum(1).mean()
    (lc * (scale * nu)).backward()
    np.testing.assert_allclose(loss.item(), lc.item(), rtol=1e-5)
    torch.testing.assert_close(dz0, a.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(dz1, b.grad, rtol=1e-4, atol=1e-6)


def test_comatch_focal_fwd_bwd():
    torch.manual_seed(9)
    nu, C, scale = 448, 23, 2.0 / 448
    ls = torch.randn(nu, C, device=DEV) * 3
    probs = torch.softmax(torch.randn(nu, C, device=DEV) * 3, -1) * 0.9  # rows sum to alpha (empty bank)
    mask = (torch.rand(nu, device=DEV) > 0.4).float()
    loss, dls = torch.zeros(1, device=DEV), torch.zeros(nu, C, device=DEV)
    ws = torch.zeros(nu, device=DEV)
    call("es_comatch_focal_fwd_bwd", ptr(ls), C, ptr(probs), ptr(mask), nu, C, 2.0, scale, ptr(loss), ptr(dls), C,
         ptr(ws), S())
    lr = ls.clone().requires_grad_(True)
    logp = -torch.sum(F.log_softmax(lr, dim=1) * probs, dim=1) * mask  # code/comatch.py:216-220
    p = torch.exp(-logp)
    lu = ((1 - p) ** 2 * logp).mean()
    (lu * (scale * nu)).backward()
    np.testing.assert_allclose(loss.item(), lu.item(), rtol=1e-5)
    torch.testing.assert_close(dls, lr.grad, rtol=1e-4, atol=1e-7)


def test_dropout_keep_mask():
    n = 1 << 20
    a, b = torch.zeros(n, dtype=torch.uint8, device=DEV), torch.zeros(n, dtype=torch.uint8, device=DEV)
    call("es_dropout_keep", ptr(a), n, 0.2, 7, 0, S())
    call("es_dropout_keep", ptr(b), n, 0.2, 7, 0, S())
    assert torch.equal(a, b)  # reproducible for (seed, offset)
    frac = a.float().mean().item()
    assert abs(frac - 0.8) < 3e-3, frac
    call("es_dropout_keep", ptr(b), n, 0.2, 7, n, S())
    assert not torch.equal(a, b)


# ------------------------------------------------------------------------------------- trainer
class _DL:
    def __init__(self, items, df=None):
        self.items = items

        class _DS:
            pass

        self.dataset = _DS()
        self.dataset.df = df

    def __iter__(self):
        return iter(self.items)

    def __len__(self):
        return len(self.items)


def _cfg(thres, steps, B, MU, L):
    from endossl.utils import AttrDict
    return AttrDict(
        DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=64, TARGET_NAME="target"),
        MODEL=AttrDict(NAME="vit_tiny_test", NUM_CLASSES=23, MARGIN="None", TYPE_SEMI="CoMatch", LOW_DIM=L),
        TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=steps, CLS_WEIGHT=False,
                       THRES=thres, T=1.0, LAMBDA_U=2.0, LAMBDA_C=2.0, IS_SSL=True, EPOCHS=1, WARMUP_EPOCHS=0,
                       DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const", FREQ_EVAL=1))


@pytest.mark.parametrize("tag", ["open", "closed"])
def test_comatch_trainer_vs_reference_train_one(golden, tag):
    """CoMatch.step against the reference (code/comatch.py:133-235).

    Step 0, tight: every stage after the trunk is checked against the oracle evaluated on the HIP
    path's OWN inputs to that stage (trunk features -> heads -> DA / smoothing / pseudo-labels ->
    losses -> d(loss)/d(logits, z) -> heads backward), fp32 against fp32.  The trunk features are
    held to the bf16-contract emulation.
    Both steps, trajectory: logits, losses, DA history, bank, BN buffers and parameters against the
    reference fixture within the bf16 envelope (the oracle's bf16-contract run vs the fixture):
    BatchNorm1d over n = 14 rows and exp(z.z / 0.2) amplify bf16 trunk noise, so the envelope, not a
    fixed 1e-3, is the meaningful bar after the first update."""
    from endossl.comatch import CoMatch
    from endossl.comatch_model import NativeViTEmb
    from endossl.vit import ViTConfig
    d = golden(f"comatch_step_{tag}.npz")
    L, steps, B, MU = int(d["L"]), int(d["steps"]), int(d["B"]), int(d["MU"])
    thres = float(d["thres"])
    rcfg = ref.Cfg(img_size=64, patch=16, dim=128, depth=2, heads=2, num_classes=23)
    vcfg = ViTConfig(img_size=64, dim=128, depth=2, heads=2, num_classes=23, head="emb", low_dim=L)
    names = [n for n, _ in ref.emb_param_shapes(rcfg, L)]
    params = {n: torch.tensor(d["init/" + n]) for n in names}
    bufs = {n: torch.tensor(d["init/" + n]) for n in ref.BN_BUFFERS}
    m = NativeViTEmb(vcfg, seed=0)
    assert list(m.state_dict().keys()) == [k[5:] for k in d.files if k.startswith("init/")]  # ModelwEmb names/order
    m.load_state_dict({**params, **bufs})
    m = m.to(DEV)
    tr = CoMatch(m, opt_func="Adam", lr=1e-3, device=DEV)
    tr.queue_batch = int(d["queue_batch"])
    lab = (torch.tensor(d["x0"]), torch.tensor(d["y0"]))  # fresh labeled iterator every step (reference)
    unl = [((torch.tensor(d[f"uw{i}"]), torch.tensor(d[f"us0_{i}"]), torch.tensor(d[f"us1_{i}"])), None)
           for i in range(steps)]
    tr.get_dataloader((_DL([lab]), _DL(unl)), None)
    tr.get_config(_cfg(thres, steps, B, MU, L))
    assert tr.queue_size == int(d["queue_size"])
    mk = lambda bf: ref.CoMatchRef(params, bufs, rcfg, L, 23, int(d["queue_size"]), thres=thres,  # noqa: E731
                                   lambda_u=2.0, lambda_c=2.0, bf16=bf)
    emu, f32, stage = mk(True), mk(False), mk(False)
    stage.queue_feats, stage.queue_probs = stage.queue_feats.clone(), stage.queue_probs.clone()
    bt, btu = B, B * MU
    rec = {}
    for i in range(steps):
        keep = torch.tensor(d[f"dropmask{i}"])
        o = tr.step((lab, unl[i]), drop_keep=keep)
        torch.cuda.synchronize()
        imgs = unl[i][0]
        r = emu.step(*lab, *imgs, keep)
        f32.step(*lab, *imgs, keep)
        lg, lg16, lg32 = o["logits"].detach().cpu().double(), r["logits"].double(), torch.tensor(d[f"logits{i}"]).double()
        env = (lg16 - lg32).abs().max().item()
        err = (lg - lg32).abs().max().item()
        sc = max(1.0, lg32.abs().max().item())
        rec[f"step{i}_logits"] = {"hip_vs_ref": err, "bf16_envelope": env}
        if i == 0:
            # trunk: CLS features vs the bf16-contract emulation (the final LayerNorm divides by each
            # row's std, so single operand-rounding flips show at ~1e-3 relative)
            f_hip = o["fts"].detach().cpu().double()
            f16, f32_ = r["fts"].double(), torch.tensor(d["fts0"]).double()
            fsc, fenv = max(1.0, f16.abs().max().item()), (f16 - f32_).abs().max().item()
            rec["step0_fts_vs_bf16_contract"] = (f_hip - f16).abs().max().item()
            rec["step0_fts_bf16_envelope"] = fenv
            assert rec["step0_fts_vs_bf16_contract"] <= 1e-3 * fsc + 0.25 * fenv, rec
            # heads on the HIP features (fp32 vs fp32)
            hp = {k: params[k].clone().requires_grad_(True) for k in names if k.startswith(("fc.", "head_emb."))}
            fts_leaf = o["fts"].detach().cpu().float().requires_grad_(True)
            lg_h, z_h = ref.emb_heads(hp, {k: v.clone() for k, v in bufs.items()}, fts_leaf, keep, train=True)
            rec["step0_heads_vs_oracle"] = (lg - lg_h.double()).abs().max().item()
            assert rec["step0_heads_vs_oracle"] <= 1e-4 * sc, rec
            torch.testing.assert_close(o["z"].detach().cpu(), z_h.detach(), rtol=1e-4, atol=1e-5)
            # DA / smoothing / pseudo-labels / losses on the HIP logits and z
            lg_leaf = o["logits"].detach().cpu().float().requires_grad_(True)
            z_leaf = o["z"].detach().cpu().float().requires_grad_(True)
            rs = stage.losses(lg_leaf, z_leaf, lab[1], bt, btu)
            for k in ("lx", "lu", "lc", "loss"):
                rec[f"step0_{k}_vs_oracle"] = [o[k].item(), rs[k]]
                assert abs(o[k].item() - rs[k]) <= 1e-4 * max(1.0, abs(rs[k])), (k, o[k].item(), rs[k])
            torch.testing.assert_close(o["probs_orig"].cpu(), rs["probs_orig"], rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(o["probs"].cpu(), rs["probs"], rtol=1e-5, atol=1e-6)
            p = rs["probs"].double()
            top2 = p.topk(2, -1).values
            ok = ((top2[:, 0] - top2[:, 1]) > 1e-5).numpy()
            okm = ((p.max(-1).values - thres).abs() > 1e-5).numpy()
            np.testing.assert_array_equal(o["pseudo_label"].cpu().numpy()[ok], rs["pseudo_label"].numpy()[ok])
            np.testing.assert_array_equal(o["mask"].cpu().numpy().astype(bool)[okm], rs["mask"].numpy().astype(bool)[okm])
            rec["step0_mask"] = o["mask"].cpu().tolist()
            hist0 = torch.stack(tr.prob_list).cpu()
            torch.testing.assert_close(hist0, torch.stack(stage.prob_list), rtol=1e-5, atol=1e-7)
            # d(loss)/d(logits, z) and the heads backward on the HIP features
            rs["loss_t"].backward()
            W = tr._workspace(bt, btu, 23, L)
            torch.testing.assert_close(W["dl"].cpu(), lg_leaf.grad, rtol=1e-4, atol=1e-6)
            torch.testing.assert_close(W["dz"].cpu(), z_leaf.grad, rtol=1e-4, atol=1e-6)
            torch.autograd.backward([lg_h, z_h], [lg_leaf.grad, z_leaf.grad])
            dfts = m.heads().bufs(bt + 3 * btu)["dfts"].cpu()
            torch.testing.assert_close(dfts, fts_leaf.grad, rtol=1e-4, atol=1e-5)
            eng = m.engine()
            for k, v in hp.items():
                torch.testing.assert_close(eng.view(m.flat_grad, k).cpu().view(v.shape), v.grad, rtol=1e-4, atol=1e-5,
                                           msg=lambda s, k=k: f"{k}: {s}")
        assert err <= 1.5 * env + 1e-3 * sc, (i, err, env)
        for k, ref_v in (("lx", float(d["lx"][i])), ("loss", float(d["loss"][i]))):
            hip, em = o[k].item(), r[k]
            s2 = max(1.0, abs(ref_v))
            rec[f"step{i}_{k}"] = {"hip": hip, "reference": ref_v, "bf16_contract": em}
            assert abs(hip - ref_v) <= 1.5 * abs(em - ref_v) + 1e-3 * s2, (i, k, hip, ref_v, em)
    # trajectory: DA history, bank and BN buffers against the fixture within the bf16 envelope
    hist, hist_ref = torch.stack(tr.prob_list).cpu(), torch.tensor(d["prob_list"])
    henv = (torch.stack(emu.prob_list) - hist_ref).abs().max().item()
    assert (hist - hist_ref).abs().max().item() <= 1.5 * henv + 1e-3, ((hist - hist_ref).abs().max(), henv)
    assert tr.queue_ptr == int(d["queue_ptr"])
    if tag == "open":
        for mine, theirs, key in ((tr.queue_feats, emu.queue_feats, "queue_feats"), (tr.queue_probs, emu.queue_probs,
                                                                                    "queue_probs")):
            fx = torch.tensor(d[key])
            e, ev = (mine.cpu() - fx).abs().max().item(), (theirs - fx).abs().max().item()
            assert e <= 1.5 * ev + 2e-3, (key, e, ev)
    else:
        assert torch.count_nonzero(tr.queue_feats) == 0
    sd, esd = m.state_dict(), tr.ema_model.ema.state_dict()
    worst, worst_e = 0.0, 0.0
    for n in names:
        if ("final/" + n) in d.files:
            worst = max(worst, (sd[n].cpu() - torch.tensor(d["final/" + n])).abs().max().item())
            worst_e = max(worst_e, (esd[n].cpu() - torch.tensor(d["ema/" + n])).abs().max().item())
        else:
            assert abs(sd[n].double().sum().item() - float(d["final_sum/" + n])) <= (2e-3 * steps + 1e-5) * sd[n].numel()
    for n in ref.BN_BUFFERS:  # running stats follow the batch statistics of the (bf16-trunk) features
        key = ("final/" + n) if ("final/" + n) in d.files else None
        if n.endswith("num_batches_tracked"):
            assert int(sd[n].item()) == steps
        elif key:
            fx = torch.tensor(d[key])
            e, ev = (sd[n].cpu() - fx).abs().max().item(), (emu.bufs[n] - fx).abs().max().item()
            assert e <= 1.5 * ev + 2e-3, (n, e, ev)
    rec["max_param_delta"], rec["max_ema_delta"] = worst, worst_e
    print(json.dumps(rec))
    assert worst <= 2e-3 * steps + 1e-5
    assert worst_e <= 1e-3 * 2e-3 * steps * (steps + 1) / 2 + 1e-6


def test_comatch_bank_resize_between_steps():
    """set_queue_size after a step (the C1 65,536-entry bank is set this way): the pseudo-label
    workspace is sized by the queue size, so it must be re-made -- a step at the larger bank runs,
    smooths against the new bank and writes into it without touching memory past its end."""
    from endossl.comatch import CoMatch
    from endossl.comatch_model import NativeViTEmb
    from endossl.vit import ViTConfig
    L, B, MU = 16, 2, 2
    m = NativeViTEmb(ViTConfig(img_size=64, dim=128, depth=2, heads=2, num_classes=23, head="emb", low_dim=L),
                     seed=3).to(DEV)
    tr = CoMatch(m, opt_func="Adam", lr=1e-3, device=DEV)
    g = torch.Generator().manual_seed(9)
    batches = [((torch.randn(B, 3, 64, 64, generator=g), torch.randint(0, 23, (B,), generator=g)),
                (tuple(torch.randn(B * MU, 3, 64, 64, generator=g) for _ in range(3)), None)) for _ in range(3)]
    tr.get_dataloader((_DL([b[0] for b in batches]), _DL([b[1] for b in batches])), None)
    tr.get_config(_cfg(0.3, 3, B, MU, L))
    tr.step(batches[0])
    q0 = tr.queue_size
    tr.set_queue_size(4 * q0 + 64)
    guard = torch.full((1 << 20,), 7.0, device=DEV)  # allocated after the resize: a stale workspace would be
    out = tr.step(batches[1])                         # smaller than the new bank's and overrun such blocks
    torch.cuda.synchronize()
    assert torch.isfinite(out["loss"]).item() and torch.all(guard == 7.0)
    assert tr.queue_feats.shape[0] == 4 * q0 + 64
    # a bank of exactly the batch's rows opens the reference's write gate (code/comatch.py:192)
    n = B + B * MU
    tr.set_queue_size(n)
    out = tr.step(batches[2])
    torch.cuda.synchronize()
    assert torch.isfinite(out["loss"]).item() and torch.all(guard == 7.0)
    assert tr.queue_ptr == 0 and tr.queue_feats.abs().sum(1).gt(0).all().item()
    norms = tr.queue_feats.norm(dim=1)
    torch.testing.assert_close(norms, torch.ones_like(norms), rtol=1e-4, atol=1e-4)  # L2-normalised z rows
