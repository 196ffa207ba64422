"""Supervised trainer with the reference's API (`SupLearning`, code/supervised.py:23-360) over the
native models -- BASELINE configs[0] (ResNet-18, 23 classes, B=16, 224²) as a GPU step.

Same constructor and methods -- get_dataloader(train_dl, valid_dl, mixup_fn, test_dl), get_config,
train_one, evaluate_one, save_checkpoint, load_checkpoint, fit -- plus `step(batch)`.  One step
(:111-138, the plain path: MODEL.MARGIN 'None', no triplet, no mixup):

  fwd    logits = model(images)
  loss   F.cross_entropy(logits, y, weight=class_weights, reduction='mean')   (ce_loss type 'none',
         code/loss.py:118) -- value and d(loss)/d(logits) in one kernel (es_ce_weighted_fwd_bwd)
  bwd    autograd over the HIP ops
  opt    Adam + EMA of the parameters in one sweep, EMA of the BatchNorm buffers, LR update

The margin (AngularPenaltySMLoss), triplet and mixup paths are out of the §8 scope
and raise NotImplementedError.
"""
import os
from datetime import date, datetime

import numpy as np
import torch

from . import _lib, dist
from ._lib import call, ptr
from .conformer import join_wgrad_stream
from .ema import ModelEMA
from .loss import weighted_ce_fwd_bwd
from .lr_scheduler import build_scheduler
from .optimizer import build_optimizer
from .throttle import StepThrottle
from .utils import AverageMeter, balanced_class_weights, calculate_metrics


class SupLearning:
    def __init__(self, model, opt_func="Adam", lr=1e-3, device='cpu', wandb=None):
        self.model = model
        self.opt_func = opt_func
        self.device = device
        self.model.to(self.device)
        self.epoch_start = 0
        self.best_valid_loss = None
        self.best_valid_score = None
        self.wandb = wandb
        self._inflight = StepThrottle()

    def get_dataloader(self, train_dl, valid_dl, mixup_fn=None, test_dl=None):
        self.train_dl = train_dl
        self.valid_dl = valid_dl
        self.test_dl = test_dl
        if mixup_fn is not None:
            raise NotImplementedError("mixup (code/supervised.py:112-113) is outside the native step's scope")
        self.mixup_fn = None

    def get_config(self, config):
        self.config = config
        print('Training mode: Supervised Learning')
        if getattr(config.MODEL, "IS_TRIPLET", False) or str(getattr(config.MODEL, "MARGIN", "None")) != "None":
            raise NotImplementedError("the triplet / angular-margin losses are outside the native step's scope")
        dist.broadcast_(self.model.flat)
        self.model.mark_updated()
        self.ema_model = ModelEMA(model=self.model, decay=config.TRAIN.EMA_DECAY, device=self.device) \
            if config.TRAIN.USE_EMA else None
        self.optimizer = build_optimizer(self.model, opt_func=self.opt_func, lr=config.TRAIN.BASE_LR)
        n_iter = len(self.train_dl) if self.train_dl is not None else 1
        self.lr_scheduler = build_scheduler(config=config, optimizer=self.optimizer, n_iter_per_epoch=n_iter)
        if config.TRAIN.CLS_WEIGHT:
            df = self.train_dl.dataset.df
            self.class_weights = torch.tensor(balanced_class_weights(df[config.DATA.TARGET_NAME]),
                                              dtype=torch.float).to(self.device)
        else:
            self.class_weights = None

    # The forward / loss / backward of a step as one hipGraph (torch.cuda.CUDAGraph over the C-ABI launches,
    # the conv weight-gradient side stream forked and joined inside): ResNet-18 at B=16 is host-bound eager
    # (Python autograd walks ~250 launches a step).  Captured after GRAPH_WARM eager steps of a shape (the
    # first versions build the conv-weight pack table; the captured step packs in one launch), then
    # replayed; inputs are copied into the graph's own buffers.  The optimizer, EMA and LR schedule stay
    # outside (their scalars change per step).  One process only: at world > 1 the weighted loss
    # all-reduces inside the step.  ENDOSSL_SUP_GRAPH=0 keeps every step eager.
    use_graph = os.environ.get("ENDOSSL_SUP_GRAPH", "1") == "1"
    GRAPH_WARM = 2

    def _compute(self, images, targets):
        """Forward, weighted CE and its gradient, backward into model.flat_grad (no host sync)."""
        dev = self.model.flat.device
        logits = self.model(images)
        stats = torch.zeros(1, dtype=torch.float32, device=dev)
        dl = torch.empty_like(logits)
        weighted_ce_fwd_bwd(logits.detach(), targets, self.class_weights, dl, stats)
        self.optimizer.zero_grad()
        torch.autograd.backward([logits], [dl])
        join_wgrad_stream(dev)
        return stats, logits.detach()

    def _graph_key(self, images, targets):
        """Everything that changes the captured launch sequence: shapes, buffers, the model's precision / map /
        freezing state and which parameters take gradients."""
        m = self.model
        cw = self.class_weights
        return (tuple(images.shape), images.dtype, tuple(targets.shape), m.flat.data_ptr(), m.flat_grad.data_ptr(),
                cw.data_ptr() if cw is not None else 0, getattr(m, "conv_bf16", None), getattr(m, "map_bf16", None),
                bool(getattr(m, "frozen_trunk", False)), tuple(p.requires_grad for p in m.parameters()))

    def _run_graph(self, images, targets):
        """One step replayed from the graph captured for its key (one graph per key, so the smaller last batch
        of an epoch runs eagerly / gets its own graph without discarding the main one).  Returns fresh copies
        of the graph's static outputs: the next replay overwrites them."""
        key = self._graph_key(images, targets)
        graphs = self.__dict__.setdefault("_graphs", {})
        ent = graphs.get(key)
        if ent is None:
            ent = graphs[key] = {"warm": 0, "graph": None}
        if ent["graph"] is None:
            if ent["warm"] < self.GRAPH_WARM:
                ent["warm"] += 1
                return self._compute(images, targets)
            gin = (images.clone(), targets.clone())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                gout = self._compute(*gin)
            ent.update(graph=g, gin=gin, gout=gout)
        else:
            for dst, src in zip(ent["gin"], (images, targets)):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src, non_blocking=True)
        ent["graph"].replay()
        return tuple(t.clone() for t in ent["gout"])

    def step(self, batch):
        """batch = (images [n, 3, H, W], targets [n]) -> {"loss", "logits"} (device tensors)."""
        images, targets = batch
        dev = self.model.flat.device
        self._inflight.wait()
        targets = targets.to(dev, non_blocking=True).to(torch.int64).contiguous()
        images = images.to(dev, non_blocking=True)
        self.model.train()
        # graph replay for the ResNet models (the host-bound P0 step); the ViT models step eagerly here
        if self.use_graph and dist.world_size() == 1 and images.is_cuda and type(self.model).__name__ == "NativeResNet":
            stats, logits = self._run_graph(images, targets)
        else:
            stats, logits = self._compute(images, targets)
        gscale = dist.allreduce_sum_(self.model.flat_grad)
        ema = self.ema_model
        self.optimizer.step(ema_flat=ema.ema.flat if ema is not None else None,
                            ema_decay=float(ema.decay) if ema is not None else 0.0, grad_scale=gscale)
        if ema is not None:
            ema.update_buffers(self.model)
            ema.ema.mark_updated()
        self._inflight.record()
        return {"loss": stats[0], "logits": logits.detach()}

    def train_one(self, epoch):
        self.model.train()
        summary_loss = AverageMeter()
        num_steps = len(self.train_dl)
        pending = []
        for step, batch in enumerate(self.train_dl):
            out = self.step(batch)
            self.lr_scheduler.step_update(epoch * num_steps + step)
            pending.append(out["loss"].detach().clone())
        for v in pending:  # one host sync per epoch
            summary_loss.update(v.item(), self.config.DATA.BATCH_SIZE)
        return summary_loss

    def evaluate_one(self, epoch=None, show_metric=False, show_report=False, show_cf_matrix=False):
        """code/supervised.py:148-196: unweighted CE mean, prediction = argmax softmax(logits)."""
        eval_model = self.ema_model.ema if self.config.TRAIN.USE_EMA else self.model
        eval_model.eval()
        summary_loss = AverageMeter()
        outs, tgts = [], []
        dev = self.model.flat.device
        with torch.no_grad():
            for images, targets in self.valid_dl:
                logits = eval_model(images.to(dev))
                targets = targets.to(dev).to(torch.int64).contiguous()
                st = torch.zeros(1, device=dev)
                scratch = torch.empty_like(logits)
                call("es_ce_weighted_fwd_bwd", ptr(logits), logits.shape[1], ptr(targets), None, logits.shape[0],
                     logits.shape[1], 1.0, ptr(scratch), logits.shape[1], ptr(st), _lib.stream())
                summary_loss.update(st.item(), self.config.DATA.BATCH_SIZE)
                outs.append(logits.argmax(1).cpu().numpy())
                tgts.append(targets.cpu().numpy())
        pred, tgt = np.concatenate(outs), np.concatenate(tgts)
        metric = calculate_metrics(pred, tgt, self.config)
        if show_metric:
            print('Metric:')
            print(metric)
        if show_report:
            from sklearn.metrics import classification_report
            print(classification_report(tgt, pred))
        return summary_loss, metric

    def save_checkpoint(self, foldname):
        """Same dict keys and filename scheme as code/supervised.py:271-293."""
        checkpoint = {}
        if self.config.TRAIN.USE_EMA:
            checkpoint['ema_state_dict'] = self.ema_model.ema.state_dict()
        d = date.today().strftime("%m_%d_%Y")
        h = datetime.now().strftime("%H_%M_%S").split('_')
        h[0] = str(int(h[0]) + 2)
        filename = d + '_' + '_'.join(h) + '_epoch_' + str(self.epoch)
        checkpoint['epoch'] = self.epoch
        checkpoint['best_valid_loss'] = self.best_valid_loss
        checkpoint['best_valid_score'] = self.best_valid_score
        checkpoint['model_state_dict'] = self.model.state_dict()
        checkpoint['optimizer'] = self.optimizer.state_dict()
        checkpoint['scheduler'] = self.lr_scheduler.state_dict()
        f = os.path.join(foldname, filename + '.pth')
        torch.save(checkpoint, f)
        return f

    def load_checkpoint(self, checkpoint_dir, is_train=False):
        checkpoint = torch.load(checkpoint_dir, map_location='cpu', weights_only=True)
        self.model.load_state_dict(checkpoint['model_state_dict'])
        for p in self.model.parameters():
            p.requires_grad = bool(is_train)
        if self.config.TRAIN.USE_EMA:
            self.ema_model.ema.load_state_dict(checkpoint['ema_state_dict'])
        self.epoch_start = checkpoint['epoch']
        self.optimizer.load_state_dict(checkpoint['optimizer'])
        self.lr_scheduler.load_state_dict(checkpoint['scheduler'])

    def fit(self):
        count_early_stop = 0
        for epoch in range(self.epoch_start, self.config.TRAIN.EPOCHS):
            if count_early_stop > 5:
                print('Early stopping')
                break
            self.epoch = epoch
            train_loss = self.train_one(self.epoch)
            print(f'\tTrain Loss: {train_loss.avg:.3f}')
            if epoch % self.config.TRAIN.FREQ_EVAL == 0 and self.valid_dl is not None:
                valid_loss, valid_metric = self.evaluate_one(self.epoch)
                f1 = float(valid_metric['macro/f1'])
                # code/supervised.py:344-358: save on a better loss AND score, count the epochs that
                # are worse in either (never reset, as in the reference)
                if self.best_valid_loss and self.best_valid_score:
                    if self.best_valid_loss > valid_loss.avg and self.best_valid_score < f1:
                        self.best_valid_loss, self.best_valid_score = valid_loss.avg, f1
                        if dist.rank() == 0:
                            self.save_checkpoint(self.config.TRAIN.SAVE_CP)
                    elif self.best_valid_loss < valid_loss.avg or self.best_valid_score > f1:
                        count_early_stop += 1
                else:
                    self.best_valid_loss, self.best_valid_score = valid_loss.avg, f1
                    if dist.rank() == 0:
                        self.save_checkpoint(self.config.TRAIN.SAVE_CP)
                print(f'\tValid Loss: {valid_loss.avg:.3f}')
                print(f'\tMetric: {valid_metric}')
