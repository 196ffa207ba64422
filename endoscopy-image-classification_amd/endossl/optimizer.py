"""build_optimizer (code/optimizer.py:29-53) for the native model: Adam(betas=(0.9, 0.999),
eps=1e-8, weight_decay=0) over the flat parameter buffer, one HBM sweep per step, optionally fused
with the EMA update (es_adam_ema_step).  The reference's two param groups (set_weight_decay,
code/optimizer.py:13-27) are kept as views for scheduler / checkpoint compatibility; with wd=0
they are numerically identical.  TRAIN.WEIGHT_DECAY is ignored, as in the reference
(SURVEY.md Appendix A.8).
"""
import math

import torch

from . import _lib
from ._lib import call, ptr


class NativeAdam:
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.model = model
        self.betas, self.eps = betas, eps
        self.param_groups = [{"lr": lr, "initial_lr": lr, "weight_decay": 0.0, "name": "decay"},
                             {"lr": lr, "initial_lr": lr, "weight_decay": 0.0, "name": "no_decay"}]
        self.exp_avg = torch.zeros_like(model.flat)
        self.exp_avg_sq = torch.zeros_like(model.flat)
        self.step_count = 0

    def zero_grad(self, set_to_none=False):
        self.model.flat_grad.zero_()

    def step(self, ema_flat=None, ema_decay=0.999, grad_scale=1.0):
        """One Adam update from model.flat_grad (x grad_scale); fused EMA if ema_flat is given."""
        if self.exp_avg.device != self.model.flat.device:
            self.exp_avg = self.exp_avg.to(self.model.flat.device)
            self.exp_avg_sq = self.exp_avg_sq.to(self.model.flat.device)
        self.step_count += 1
        b1, b2 = self.betas
        lr = self.param_groups[0]["lr"]
        # torch.optim.Adam (single-tensor): step_size = lr / bias_correction1, computed in double
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        step_size = lr / bc1
        bc2_sqrt = math.sqrt(bc2)
        p, g = self.model.flat, self.model.flat_grad
        call("es_adam_ema_step", ptr(p), ptr(g), ptr(self.exp_avg), ptr(self.exp_avg_sq), ptr(ema_flat), p.numel(),
             float(b1), float(b2), float(self.eps), float(-step_size), float(bc2_sqrt), float(ema_decay),
             float(1.0 - ema_decay), float(grad_scale), _lib.stream())
        self.model.mark_updated()

    def state_dict(self):
        return {"state": {"step": self.step_count, "exp_avg": self.exp_avg.detach().cpu(),
                          "exp_avg_sq": self.exp_avg_sq.detach().cpu()},
                "param_groups": [dict(g) for g in self.param_groups]}

    def load_state_dict(self, sd):
        st = sd["state"]
        self.step_count = int(st["step"])
        self.exp_avg.copy_(st["exp_avg"])
        self.exp_avg_sq.copy_(st["exp_avg_sq"])
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)


def build_optimizer(model, opt_func='Adam', lr=1e-3):
    opt_lower = opt_func.lower()
    if opt_lower == 'adam':
        if not hasattr(model, "flat"):
            raise NotImplementedError("native Adam needs a NativeViT (flat parameter buffer)")
        return NativeAdam(model, lr=lr)
    raise NotImplementedError(f"optimizer {opt_func!r}: only Adam (the SSL configs' choice) is native")
