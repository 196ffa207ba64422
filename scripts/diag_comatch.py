"""Diagnostic: CoMatch trainer DA history vs torch recomputation from the HIP logits (2 steps)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "endoscopy-image-classification_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from test_gpu_comatch import _DL, _cfg
from oracle import ref
from endossl.comatch import CoMatch
from endossl.comatch_model import NativeViTEmb
from endossl.vit import ViTConfig
d = np.load(os.path.join(ROOT, "tests/golden/comatch_step_closed.npz"))
L, steps, B, MU = int(d["L"]), int(d["steps"]), int(d["B"]), int(d["MU"])
rcfg = ref.Cfg(img_size=64, patch=16, dim=128, depth=2, heads=2, num_classes=23)
vcfg = ViTConfig(img_size=64, dim=128, depth=2, heads=2, num_classes=23, head="emb", low_dim=L)
names = [n for n, _ in ref.emb_param_shapes(rcfg, L)]
m = NativeViTEmb(vcfg, seed=0)
m.load_state_dict({**{n: torch.tensor(d["init/" + n]) for n in names}, **{n: torch.tensor(d["init/" + n]) for n in ref.BN_BUFFERS}})
m = m.to("cuda")
tr = CoMatch(m, device="cuda")
lab = (torch.tensor(d["x0"]), torch.tensor(d["y0"]))
unl = [((torch.tensor(d[f"uw{i}"]), torch.tensor(d[f"us0_{i}"]), torch.tensor(d[f"us1_{i}"])), None) for i in range(steps)]
tr.get_dataloader((_DL([lab]), _DL(unl)), None)
tr.get_config(_cfg(float(d["thres"]), steps, B, MU, L))
for i in range(steps):
    o = tr.step((lab, unl[i]), drop_keep=torch.tensor(d[f"dropmask{i}"]))
    torch.cuda.synchronize()
    lw = o["logits"][B:B + B * MU].float()
    pm = torch.softmax(lw, 1).mean(0).cpu()
    print(i, "pos", tr._hist_pos, "len", tr._hist_len, "logits vs fixture", (o["logits"].cpu() - torch.tensor(d[f"logits{i}"])).abs().max().item())
    print("  torch mean(softmax(lw)) vs fixture row", (pm - torch.tensor(d["prob_list"][i])).abs().max().item())
    print("  hist rows vs fixture row i:", [(tr.prob_hist[j].cpu() - torch.tensor(d["prob_list"][i])).abs().max().item() for j in range(3)])

# ---- per-tensor gradient check of step 0 against the fp32 oracle (fresh model)
m2 = NativeViTEmb(vcfg, seed=0)
params = {n: torch.tensor(d["init/" + n]) for n in names}
bufs = {n: torch.tensor(d["init/" + n]) for n in ref.BN_BUFFERS}
m2.load_state_dict({**params, **bufs})
m2 = m2.to("cuda")
tr2 = CoMatch(m2, device="cuda")
tr2.get_dataloader((_DL([lab]), _DL(unl)), None)
tr2.get_config(_cfg(float(d["thres"]), steps, B, MU, L))
r32 = ref.CoMatchRef(params, bufs, rcfg, L, 23, int(d["queue_size"]), thres=float(d["thres"]), lambda_u=2.0, lambda_c=2.0)
for ov in (True,):
    o = tr2.step((lab, unl[0]), drop_keep=torch.tensor(d["dropmask0"]))
    torch.cuda.synchronize()
    rr = r32.step(*lab, *unl[0][0], torch.tensor(d["dropmask0"]))
    eng = m2.engine()
    print("losses hip", {k: round(o[k].item(), 5) for k in ("lx", "lu", "lc", "loss")}, "ref", {k: round(rr[k], 5) for k in ("lx", "lu", "lc", "loss")})
    for n in names:
        gh = eng.view(m2.flat_grad, n).cpu().view(rr["grads"][n].shape)
        gr = rr["grads"][n]
        rel = ((gh - gr).norm() / (gr.norm() + 1e-12)).item()
        if rel > 0.05:
            print(f"  GRAD {n}: rel err {rel:.3g}  |ref| {gr.norm():.3g} |hip| {gh.norm():.3g}")
    print("grad check done")
