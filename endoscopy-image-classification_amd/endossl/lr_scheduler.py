"""build_scheduler (code/lr_scheduler.py:14-64): host-side LR scalars updated per step via
`step_update(epoch * EVAL_STEP + batch_idx)` (code/fixmatch.py:124).

timm 0.5.4's StepLRScheduler / CosineLRScheduler (and the reference's own LinearLRScheduler,
code/lr_scheduler.py:67-116) are restated here because timm is not installed.  Parity of the timm
formulas is UNPINNED (no reference test or fixture covers them).  Noise is off in
every reference construction, so it is not restated.
"""
import math


class _Scheduler:
    def __init__(self, optimizer, warmup_t=0, warmup_lr_init=0.0, t_in_epochs=False):
        self.optimizer = optimizer
        for g in optimizer.param_groups:
            g.setdefault("initial_lr", g["lr"])
        self.base_values = [g["initial_lr"] for g in optimizer.param_groups]
        self.warmup_t, self.warmup_lr_init, self.t_in_epochs = warmup_t, warmup_lr_init, t_in_epochs
        if self.warmup_t:
            self.warmup_steps = [(v - warmup_lr_init) / self.warmup_t for v in self.base_values]
            self._update_groups([warmup_lr_init] * len(self.base_values))
        else:
            self.warmup_steps = [1 for _ in self.base_values]
        self.last_update = None

    def _update_groups(self, values):
        for g, v in zip(self.optimizer.param_groups, values):
            g["lr"] = v

    def _get_lr(self, t):
        raise NotImplementedError

    def step(self, epoch, metric=None):
        if self.t_in_epochs:
            self._update_groups(self._get_lr(epoch))

    def step_update(self, num_updates, metric=None):
        self.last_update = num_updates
        if not self.t_in_epochs:
            self._update_groups(self._get_lr(num_updates))

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k != "optimizer"}

    def load_state_dict(self, sd):
        self.__dict__.update(sd)


class StepLRScheduler(_Scheduler):
    def __init__(self, optimizer, decay_t, decay_rate=1.0, warmup_t=0, warmup_lr_init=0.0, t_in_epochs=True):
        self.decay_t, self.decay_rate = decay_t, decay_rate
        super().__init__(optimizer, warmup_t, warmup_lr_init, t_in_epochs)

    def _get_lr(self, t):
        if t < self.warmup_t:
            return [self.warmup_lr_init + t * s for s in self.warmup_steps]
        return [v * (self.decay_rate ** (t // self.decay_t)) for v in self.base_values]


class CosineLRScheduler(_Scheduler):
    def __init__(self, optimizer, t_initial, lr_min=0.0, cycle_mul=1.0, cycle_decay=1.0, cycle_limit=1,
                 warmup_t=0, warmup_lr_init=0.0, warmup_prefix=False, t_in_epochs=True, k_decay=1.0):
        self.t_initial, self.lr_min, self.cycle_mul, self.cycle_decay = t_initial, lr_min, cycle_mul, cycle_decay
        self.cycle_limit, self.warmup_prefix, self.k_decay = cycle_limit, warmup_prefix, k_decay
        super().__init__(optimizer, warmup_t, warmup_lr_init, t_in_epochs)

    def _get_lr(self, t):
        if t < self.warmup_t:
            return [self.warmup_lr_init + t * s for s in self.warmup_steps]
        if self.warmup_prefix:
            t = t - self.warmup_t
        if self.cycle_mul != 1:
            i = math.floor(math.log(1 - t / self.t_initial * (1 - self.cycle_mul), self.cycle_mul))
            t_i = self.cycle_mul ** i * self.t_initial
            t_curr = t - (1 - self.cycle_mul ** i) / (1 - self.cycle_mul) * self.t_initial
        else:
            i = t // self.t_initial
            t_i = self.t_initial
            t_curr = t - (self.t_initial * i)
        gamma = self.cycle_decay ** i
        k = self.k_decay
        if i < self.cycle_limit:
            return [self.lr_min + 0.5 * (v * gamma - self.lr_min) * (1 + math.cos(math.pi * t_curr ** k / t_i ** k))
                    for v in self.base_values]
        return [self.lr_min for _ in self.base_values]


class LinearLRScheduler(_Scheduler):
    """code/lr_scheduler.py:67-116 (the reference's own class)."""

    def __init__(self, optimizer, t_initial, lr_min_rate, warmup_t=0, warmup_lr_init=0.0, t_in_epochs=True):
        self.t_initial, self.lr_min_rate = t_initial, lr_min_rate
        super().__init__(optimizer, warmup_t, warmup_lr_init, t_in_epochs)

    def _get_lr(self, t):
        if t < self.warmup_t:
            return [self.warmup_lr_init + t * s for s in self.warmup_steps]
        t = t - self.warmup_t
        total_t = self.t_initial - self.warmup_t
        return [v - ((v - v * self.lr_min_rate) * (t / total_t)) for v in self.base_values]


def build_scheduler(config, optimizer, n_iter_per_epoch):
    num_steps = int(config.TRAIN.EPOCHS * n_iter_per_epoch)
    warmup_steps = int(config.TRAIN.WARMUP_EPOCHS * n_iter_per_epoch)
    decay_steps = int(config.TRAIN.DECAY_EPOCHS * n_iter_per_epoch)
    warmup_lr_init = config.TRAIN.WARMUP_LR
    name = config.TRAIN.SCH_NAME
    if name == 'cosine':
        return CosineLRScheduler(optimizer, t_initial=num_steps, cycle_mul=1., lr_min=5e-6,
                                 warmup_lr_init=warmup_lr_init, warmup_t=warmup_steps, cycle_limit=1,
                                 t_in_epochs=False)
    if name == 'linear':
        return LinearLRScheduler(optimizer, t_initial=num_steps, lr_min_rate=0.01, warmup_lr_init=warmup_lr_init,
                                 warmup_t=warmup_steps, t_in_epochs=False)
    if name == 'step':
        return StepLRScheduler(optimizer, decay_t=decay_steps, decay_rate=config.TRAIN.LR_DECAY,
                               warmup_lr_init=warmup_lr_init, warmup_t=warmup_steps, t_in_epochs=False)
    if name in ('const', 'constant', 'none'):
        return None
    raise ValueError(f"unknown SCH_NAME {name!r}")
