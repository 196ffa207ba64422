"""build_optimizer (code/optimizer.py:29-53) for the native model: Adam(betas=(0.9, 0.999),
eps=1e-8, weight_decay=0) over the flat parameter buffer, one HBM sweep per step, optionally fused
with the EMA update (es_adam_ema_step).  TRAIN.WEIGHT_DECAY is ignored, as in the reference
(SURVEY.md Appendix A.8).

Checkpoints use torch.optim.Adam's own state_dict format, so a native checkpoint resumes in the
reference and the other way round: the two param groups of set_weight_decay (code/optimizer.py:
13-27: trainable parameters only, in named_parameters order; 1-D tensors, `.bias` and the model's
no_weight_decay() names go to the second group), parameter indices numbered group by group, and
per-index state {'step', 'exp_avg', 'exp_avg_sq'} shaped like the parameter.  On the device the
moments stay two flat buffers in the parameter layout; frozen parameters (IS_FREEZE) get a zero
gradient and zero moments, so the fused sweep leaves them bit-for-bit unchanged.
"""
import math

import torch

from . import _lib
from ._lib import call, ptr


def _in_keywords(name, keywords):
    return any(k in name for k in keywords)


def weight_decay_groups(model):
    """(decay, no_decay) lists of parameter names, as set_weight_decay (code/optimizer.py:13-27)
    splits model.named_parameters()."""
    skip = model.no_weight_decay() if hasattr(model, "no_weight_decay") else set()
    skip_kw = model.no_weight_decay_keywords() if hasattr(model, "no_weight_decay_keywords") else set()
    decay, no_decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        if len(p.shape) == 1 or name.endswith(".bias") or name in skip or _in_keywords(name, skip_kw):
            no_decay.append(name)
        else:
            decay.append(name)
    return decay, no_decay


class NativeAdam:
    _GROUP_DEFAULTS = {"amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                       "differentiable": False, "fused": None}

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.model = model
        self.betas, self.eps = betas, eps
        decay, no_decay = weight_decay_groups(model)
        self._group_names = [decay, no_decay]
        common = dict(lr=lr, betas=tuple(betas), eps=eps, **self._GROUP_DEFAULTS)
        self.param_groups = [dict(common, weight_decay=0), dict(common, weight_decay=0.0)]
        self.exp_avg = torch.zeros_like(model.flat)
        self.exp_avg_sq = torch.zeros_like(model.flat)
        self.step_count = 0

    def _slice(self, buf, name):
        o = self.model.offs[name]
        shape = self.model.get_parameter(name).shape
        return buf[o:o + math.prod(shape)].view(shape)

    def zero_grad(self, set_to_none=False):
        self.model.flat_grad.zero_()

    def frozen_ranges(self):
        """Flat [lo, hi) ranges of the parameters outside both groups (requires_grad False)."""
        trainable = set(self._group_names[0]) | set(self._group_names[1])
        out = []
        for name, p in self.model.named_parameters():
            if name not in trainable:
                o = self.model.offs[name]
                out.append((o, o + p.numel()))
        return out

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

    # -------------------------------------------------------------- torch.optim.Adam format
    def state_dict(self):
        state, groups, idx = {}, [], 0
        for g, names in zip(self.param_groups, self._group_names):
            ids = []
            for name in names:
                if self.step_count > 0:
                    state[idx] = {"step": torch.tensor(float(self.step_count)),
                                  "exp_avg": self._slice(self.exp_avg, name).detach().cpu().clone(),
                                  "exp_avg_sq": self._slice(self.exp_avg_sq, name).detach().cpu().clone()}
                ids.append(idx)
                idx += 1
            groups.append(dict(g, params=ids))
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        groups = sd["param_groups"]
        if len(groups) != len(self._group_names):
            raise ValueError(f"optimizer state has {len(groups)} param groups, the model {len(self._group_names)}")
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        steps = set()
        for g, mine, names in zip(groups, self.param_groups, self._group_names):
            if len(g["params"]) != len(names):
                raise ValueError(f"param group sizes differ: checkpoint {len(g['params'])}, model {len(names)}")
            for idx, name in zip(g["params"], names):
                st = sd["state"].get(idx)
                if st is None:
                    continue
                self._slice(self.exp_avg, name).copy_(st["exp_avg"].reshape(self._slice(self.exp_avg, name).shape))
                self._slice(self.exp_avg_sq, name).copy_(
                    st["exp_avg_sq"].reshape(self._slice(self.exp_avg_sq, name).shape))
                steps.add(int(st["step"].item() if torch.is_tensor(st["step"]) else st["step"]))
            mine.update({k: v for k, v in g.items() if k != "params"})
        if len(steps) > 1:
            raise ValueError(f"per-parameter Adam step counts differ ({sorted(steps)}): the fused sweep keeps one")
        self.step_count = steps.pop() if steps else 0
        self.betas = tuple(self.param_groups[0]["betas"])
        self.eps = self.param_groups[0]["eps"]


def build_optimizer(model, opt_func='Adam', lr=1e-3):
    opt_lower = opt_func.lower()
    if opt_lower == 'adam':
        if not hasattr(model, "flat"):
            raise NotImplementedError("native Adam needs a native model (flat parameter buffer)")
        return NativeAdam(model, lr=lr)
    raise NotImplementedError(f"optimizer {opt_func!r}: only Adam (the SSL configs' choice) is native")
