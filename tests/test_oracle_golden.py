"""Pin the oracle (oracle/ref.py) against fixtures produced by the REFERENCE implementation
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import torch

from oracle import ref


def test_consistency_matches_reference(golden):
    for tag in ("0p7", "0p95", "median"):
        d = golden(f"consistency_{tag}.npz")
        lw = torch.tensor(d["logits_w"])
        ls = torch.tensor(d["logits_s"]).requires_grad_(True)
        loss, mm, pl, mask = ref.consistency(lw, ls, float(d["tau"]))
        loss.backward()
        assert loss.item() == float(d["loss"]), tag
        assert mm.item() == float(d["mask_mean"]), tag
        np.testing.assert_array_equal(pl.numpy(), d["pseudo_label"])
        np.testing.assert_array_equal(mask.numpy(), d["mask"])
        np.testing.assert_array_equal(ls.grad.numpy(), d["grad_logits_s"])
    # the forced tie in row 5 resolves to the FIRST max index, as torch.max does in the reference
    d = golden("consistency_0p7.npz")
    assert d["pseudo_label"][5] == 3


def test_poly_matches_reference(golden):
    for tag in ("weighted", "plain"):
        d = golden(f"poly_{tag}.npz")
        x = torch.tensor(d["logits"]).requires_grad_(True)
        w = torch.tensor(d["weights"]) if d["weights"].size else None
        loss = ref.poly_ce(x, torch.tensor(d["targets"]), w)
        loss.backward()
        np.testing.assert_allclose(loss.item(), float(d["loss"]), rtol=1e-6)
        np.testing.assert_allclose(x.grad.numpy(), d["grad_logits"], rtol=1e-5, atol=1e-7)


def test_ema_matches_reference(golden):
    d = golden("ema.npz")
    keys = sorted({k.split("/", 1)[1] for k in d.files if k.startswith("ema_before/")})
    ema = {k: torch.tensor(d["ema_before/" + k]) for k in keys}
    model = {k: torch.tensor(d["model/" + k]) for k in keys}
    ref.ema_update(ema, model, float(d["decay"]))
    for k in keys:
        np.testing.assert_array_equal(ema[k].numpy(), d["ema_after/" + k], err_msg=k)
    # int64 buffer: 0.999*1 + 0.001*2 = 1.001 truncates back to 1 -- the EMA counter never advances
    assert int(d["ema_before/1.num_batches_tracked"]) == 1 and int(d["model/1.num_batches_tracked"]) == 2
    assert int(d["ema_after/1.num_batches_tracked"]) == 1


def _tiny_cfg():
    return ref.Cfg(img_size=64, patch=16, dim=128, depth=2, heads=2, num_classes=23)


def test_fixmatch_step_matches_reference(golden):
    for tag, full in (("t0p7", True), ("t0p95", False)):
        d = golden(f"fixmatch_step_{tag}.npz")
        cfg = _tiny_cfg()
        params = {n: torch.tensor(d["init/" + n]) for n, _ in ref.param_shapes(cfg)}
        fm = ref.FixMatchRef(params, cfg, class_weights=torch.tensor(d["class_weights"]),
                             thres=float(d["thres"]), lambda_u=1.0, lr=1e-3, ema_decay=0.999)
        for i in range(int(d["steps"])):
            out = fm.step(torch.tensor(d[f"x{i}"]), torch.tensor(d[f"y{i}"]), torch.tensor(d[f"uw{i}"]),
                          torch.tensor(d[f"us{i}"]))
            np.testing.assert_allclose(out["lx"], d["lx"][i], rtol=1e-6)
            np.testing.assert_allclose(out["lu"], d["lu"][i], rtol=1e-6, atol=1e-7)
            assert out["mask_mean"] == d["mask_mean"][i]
            np.testing.assert_array_equal(out["pseudo_label"].numpy(), d["pseudo_label"][i])
        for n, _ in ref.param_shapes(cfg):
            if full:
                np.testing.assert_allclose(fm.p[n].detach().numpy(), d["final/" + n], rtol=1e-5, atol=1e-7,
                                           err_msg=n)
                np.testing.assert_allclose(fm.ema[n].numpy(), d["ema/" + n], rtol=1e-5, atol=1e-7, err_msg=n)
            else:
                np.testing.assert_allclose(fm.p[n].detach().double().sum().item(), d["final_sum/" + n],
                                           rtol=1e-5, atol=1e-5, err_msg=n)
                np.testing.assert_allclose(fm.ema[n].double().sum().item(), d["ema_sum/" + n], rtol=1e-5,
                                           atol=1e-5, err_msg=n)
        # the reference's LR scheduler saw epoch*EVAL_STEP + batch_idx, starting at epoch 1
        np.testing.assert_array_equal(d["lr_updates"], [2, 3])


def _comatch_ref(d, cfg):
    L, C = int(d["L"]), cfg.num_classes
    params = {n: torch.tensor(d["init/" + n]) for n, _ in ref.emb_param_shapes(cfg, L)}
    bufs = {n: torch.tensor(d["init/" + n]) for n in ref.BN_BUFFERS}
    return ref.CoMatchRef(params, bufs, cfg, L, C, int(d["queue_size"]), class_weights=None,
                          thres=float(d["thres"]), lambda_u=float(d["lambda_u"]), lambda_c=float(d["lambda_c"]),
                          lr=1e-3, ema_decay=0.999)


def test_comatch_step_matches_reference(golden):
    """CoMatch.train_one (code/comatch.py:133-235), two steps, bank gate closed (reference default)
    and open (queue_batch=1).  The labeled batch is the FIRST one in both steps: the reference
    calls next() on the DataLoader itself, which raises, and falls back to a fresh iterator every
    step (code/comatch.py:135-138)."""
    cfg = _tiny_cfg()
    for tag, full in (("open", True), ("closed", False)):
        d = golden(f"comatch_step_{tag}.npz")
        cm = _comatch_ref(d, cfg)
        for i in range(int(d["steps"])):
            out = cm.step(torch.tensor(d["x0"]), torch.tensor(d["y0"]), torch.tensor(d[f"uw{i}"]),
                          torch.tensor(d[f"us0_{i}"]), torch.tensor(d[f"us1_{i}"]), torch.tensor(d[f"dropmask{i}"]))
            np.testing.assert_allclose(out["logits"].numpy(), d[f"logits{i}"], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(out["fts"].numpy(), d[f"fts{i}"], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(out["z"].numpy(), d[f"z{i}"], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(out["lx"], d["lx"][i], rtol=1e-6)
            np.testing.assert_allclose(out["loss"], d["loss"][i], rtol=1e-6)
        np.testing.assert_allclose(torch.stack(cm.prob_list).numpy(), d["prob_list"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(cm.queue_feats.numpy(), d["queue_feats"], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(cm.queue_probs.numpy(), d["queue_probs"], rtol=1e-6, atol=1e-7)
        assert cm.queue_ptr == int(d["queue_ptr"])
        names = [n for n, _ in ref.emb_param_shapes(cfg, int(d["L"]))] + list(ref.BN_BUFFERS)
        for n in names:
            got = cm.p[n].detach() if n in cm.p else cm.bufs[n]
            if full:
                np.testing.assert_allclose(got.numpy(), d["final/" + n], rtol=1e-5, atol=1e-7, err_msg=n)
                np.testing.assert_allclose(cm.ema[n].numpy(), d["ema/" + n], rtol=1e-5, atol=1e-7, err_msg=n)
            else:
                np.testing.assert_allclose(got.double().sum().item(), d["final_sum/" + n], rtol=1e-5, atol=1e-5,
                                           err_msg=n)
                np.testing.assert_allclose(cm.ema[n].double().sum().item(), d["ema_sum/" + n], rtol=1e-5,
                                           atol=1e-5, err_msg=n)
        np.testing.assert_array_equal(d["lr_updates"], [2, 3])
    # the open variant actually exercises the bank: rows written in step 1, read in step 2
    assert np.abs(golden("comatch_step_open.npz")["queue_feats"]).sum() > 0
    assert np.abs(golden("comatch_step_closed.npz")["queue_feats"]).sum() == 0


def test_vit_s_param_count():
    cfg = ref.Cfg()
    n = sum(int(np.prod(s)) for _, s in ref.param_shapes(cfg))
    assert n == 21_674_519


def test_bf16_envelope():
    """The oracle's bf16 mode (the MI355X path's rounding points) stays within a few 1e-3 of the
    fp32 reference arithmetic -- the envelope the GPU parity tests are bounded by."""
    import torch
    cfg = ref.Cfg(img_size=64, patch=16, dim=128, depth=2, heads=2, num_classes=23)
    p = ref.random_params(cfg, seed=11, head_std=0.6)
    x = torch.randn(8, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        l32 = ref.vit_forward(p, x, cfg)
        l16 = ref.vit_forward(p, x, cfg, bf16=True)
    rel = (l16 - l32).abs().max().item() / l32.abs().max().item()
    assert 1e-4 < rel < 2e-2, rel


def test_bf16_rounding_is_discontinuous_at_depth():
    """Why the full-depth GPU bar is envelope-based: under the bf16 contract a 1e-7 relative nudge
    of the weights (which only flips bf16 rounding decisions) moves ViT-S logits by a sizeable
    fraction of the whole bf16-vs-fp32 envelope, while the fp32 arithmetic barely moves.  Any two
    bf16 implementations of the 12-layer step therefore agree only to within that envelope."""
    import torch
    cfg = ref.Cfg(depth=12)
    p = ref.random_params(cfg, seed=11, head_std=0.3)
    q = {k: v * (1 + 1e-7 * torch.randn(v.shape, generator=torch.Generator().manual_seed(2))) for k, v in p.items()}
    x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        a16, b16 = ref.vit_forward(p, x, cfg, bf16=True), ref.vit_forward(q, x, cfg, bf16=True)
        a32, b32 = ref.vit_forward(p, x, cfg), ref.vit_forward(q, x, cfg)
    envelope = (a16 - a32).abs().max().item()
    drift16 = (a16 - b16).abs().max().item()
    drift32 = (a32 - b32).abs().max().item()
    assert drift16 > 0.2 * envelope
    assert drift32 < 1e-3 * envelope * 10


def test_semiformer_step_matches_reference(golden):
    """SemiFormer.train_one SSL branch (code/semiformer.py:103-146) on a tiny Conformer
    (code/models/conformer.py:75-445): both heads' logits, the losses and the post-step state."""
    from oracle import conformer_ref as cr
    d = golden("semiformer_step.npz")
    cfg = cr.ConformerCfg(img_size=64, patch=16, base_channel=64, channel_ratio=1, embed_dim=128, depth=6, heads=2,
                          num_classes=23)
    state = {k[5:]: torch.tensor(d[k]) for k in d.files if k.startswith("init/")}
    r = cr.SemiFormerRef(state, cfg, class_weights=torch.tensor(d["class_weights"]).float(), thres=float(d["thres"]))
    for i in range(int(d["steps"])):
        x, y, uw, us = (torch.tensor(d[k]) for k in (f"x{i}", f"y{i}", f"uw{i}", f"us{i}"))
        o = r.step(x, y, uw, us)
        torch.testing.assert_close(o["out_conv"], torch.tensor(d[f"out_conv{i}"]), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(o["out_trans"], torch.tensor(d[f"out_trans{i}"]), rtol=1e-5, atol=1e-5)
        assert abs(o["lx"] - float(d["lx"][2 * i] + d["lx"][2 * i + 1])) < 1e-5
        assert abs(o["lu"] - float(d["lu"][2 * i] + d["lu"][2 * i + 1])) < 1e-5
        np.testing.assert_array_equal(o["pseudo_label"].numpy(), d["pseudo_label"][2 * i])
    assert 0.0 < float(d["mask_mean"][0]) < 1.0  # mixed masks: the threshold is exercised
    for k, v in r.p.items():
        if "final/" + k in d.files:
            torch.testing.assert_close(v.detach(), torch.tensor(d["final/" + k]), rtol=1e-5, atol=1e-6)
        else:
            assert abs(v.detach().double().sum().item() - float(d["final_sum/" + k])) <= 1e-5 * max(
                1.0, float(d["final_abs/" + k]))
    for k, v in r.bufs.items():
        torch.testing.assert_close(v, torch.tensor(d["final/" + k]), rtol=1e-5, atol=1e-6)
    for k in d.files:
        if k.startswith("ema/"):
            torch.testing.assert_close(r.ema[k[4:]], torch.tensor(d[k]), rtol=1e-5, atol=1e-6)
