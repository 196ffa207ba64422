"""FixMatch trainer with the reference's API (code/fixmatch.py:19-262) over the native step.

Same constructor and methods as the reference -- get_dataloader, get_config, train_one,
evaluate_one, save_checkpoint, load_checkpoint, fit -- plus `step(batch)`, the unit the
benchmark times.  One step (code/fixmatch.py:91-131):

  weak   logits_w = model(u_w)                forward only, on a second HIP stream beside the train
                                              forward (independent buffers); the reference detaches it
                                              (code/loss.py:144) and ViT rows are independent,
                                              so its backward is exactly zero
  train  logits   = model([x ; u_s])          forward with saved activations
  loss   lx = PolyCE(logits[:B], y, w)        fused value+grad kernel      (code/fixmatch.py:114)
         lu, mask = consistency(logits_w, logits[B:], tau)  fused kernel  (:116)
         losses = lx + LAMBDA_U * lu                                      (:118)
  bwd    flat grads <- explicit backward of d(losses)/d(logits)            (:122)
  comm   RCCL all-reduce of the flat grad (data-parallel only) after the backward; opt-in
         (ENDOSSL_OVERLAP_AR=1): one bucket per transformer block issued as soon as that block's
         gradients are final, beside the rest of the reverse pass (dist.GradBuckets)
  opt    Adam + EMA in one sweep, then lr_scheduler.step_update           (:123-127)

No `.item()` per step: losses stay on device and the AverageMeter is filled once per epoch.
"""
import os
from datetime import date, datetime

import numpy as np
import torch

from . import _lib, dist
from ._lib import call, ptr
from .ema import ModelEMA
from .loss import ce_loss
from .lr_scheduler import build_scheduler
from .optimizer import build_optimizer
from .throttle import StepThrottle
from .utils import AverageMeter, balanced_class_weights, calculate_metrics


def _next(it):
    return it.next() if hasattr(it, "next") else next(it)


class FixMatch:
    # bucketed all-reduce overlapped with the backward (world > 1): opt-in, ENDOSSL_OVERLAP_AR=1.  Off by
    # default: unmeasured over RCCL here (one GPU per box), and the two-rank gloo rehearsal on one GPU
    # ran 1.1-3.7 s/step with it vs 92 ms without whenever the engine's second stream was on
    # (129 ms with it off) -- DESIGN.md §6
    overlap_allreduce = os.environ.get("ENDOSSL_OVERLAP_AR", "0") == "1"

    def __init__(self, model, opt_func="Adam", lr=1e-3, device='cpu'):
        self.model = model
        self.opt_func = opt_func
        self.device = device
        self.model.to(self.device)
        self.epoch_start = 1
        self.best_valid_perf = None
        self._dlogits = None
        self._stats = None
        self._inflight = StepThrottle(2)

    def get_dataloader(self, train_dl, valid_dl, test_dl=None):
        self.train_labeled_dl, self.train_unlabeled_dl = train_dl
        self.valid_dl = valid_dl
        self.test_dl = test_dl

    def _trainable_when_frozen(self):
        """The modules IS_FREEZE keeps trainable (code/fixmatch.py:45-48: `model.fc`)."""
        return [self.model.fc]

    def get_config(self, config):
        self.config = config
        # code/fixmatch.py:40-52: IS_FREEZE trains `model.fc` only (timm ViT: the classifier head).  The
        # native step then runs both forwards in inference form (no saved activations) and the head's
        # backward alone (Engine.head_backward): the trunk gets exactly zero gradient and no update
        self.frozen = bool(config.TRAIN.IS_FREEZE)
        for p in self.model.parameters():
            p.requires_grad = not self.frozen
        if self.frozen:
            for mod in self._trainable_when_frozen():
                mod.requires_grad_(True)
        # identical replicas on every rank before the first step
        dist.broadcast_(self.model.flat)
        self.model.mark_updated()
        self.ema_model = ModelEMA(model=self.model, decay=config.TRAIN.EMA_DECAY, device=self.device) \
            if config.TRAIN.USE_EMA else None
        self.optimizer = build_optimizer(self.model, opt_func=self.opt_func, lr=config.TRAIN.BASE_LR)
        self.lr_scheduler = build_scheduler(config=config, optimizer=self.optimizer,
                                            n_iter_per_epoch=config.TRAIN.EVAL_STEP)
        if config.TRAIN.CLS_WEIGHT:
            df = self.train_labeled_dl.dataset.df
            w = balanced_class_weights(df[config.DATA.TARGET_NAME])
            self.class_weights = torch.tensor(w, dtype=torch.float).to(self.device)
        else:
            self.class_weights = None

    # ------------------------------------------------------------------ the hot step
    # The forward / losses / backward of a step as one hipGraph (torch.cuda.CUDAGraph over the C-ABI
    # launches, both HIP streams): ~600 kernel launches replayed without the host walking the
    # engine, which matters once a rank's share of the batch is small (strong scaling: 8 + 56 pairs
    # per GPU at N = 8).  Captured on the first step of a shape after one eager step; inputs are
    # copied into the graph's own static buffers (static_batch() hands them out for zero-copy use).
    # The optimizer, the all-reduce and the LR schedule stay outside (their scalars change per step).
    # Off by default (eager launches measured faster); ENDOSSL_GRAPH=1 turns capture on.
    # The grouped weight-gradient launches of a small shard (Engine.GROUP_WGRAD) are captured too: their
    # device-side problem tables are uploaded by the eager step and only read inside the graph.
    use_graph = os.environ.get("ENDOSSL_GRAPH", "0") == "1"

    def _compute(self, inputs_x, targets_x, inputs_u_w, inputs_u_s):
        """Weak forward, train forward, fused losses, backward into model.flat_grad (no host sync)."""
        cfg = self.config
        m = self.model
        eng = m.engine()
        dev = m.flat.device
        B, nu = int(inputs_x.shape[0]), int(inputs_u_w.shape[0])
        C = m.cfg.num_classes
        s = _lib.stream()
        if self._dlogits is None or self._dlogits.shape[0] != B + nu:
            self._dlogits = torch.empty(B + nu, C, dtype=torch.float32, device=dev)
            self._pl = torch.empty(nu, dtype=torch.int32, device=dev)
            self._mask = torch.empty(nu, dtype=torch.uint8, device=dev)
        stats = torch.empty(4, dtype=torch.float32, device=dev)  # lx, lu, mask_mean, total
        frozen = getattr(self, "frozen", False)
        if eng.overlap_fwd:  # weak forward on the side stream, beside the train forward
            main, side = torch.cuda.current_stream(dev), eng.side_stream((B + nu) * m.cfg.T)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                logits_w = eng.forward(m.flat, [inputs_u_w], train=False)
            logits = eng.forward(m.flat, [inputs_x, inputs_u_s], train=not frozen)
            main.wait_stream(side)
        else:
            logits_w = eng.forward(m.flat, [inputs_u_w], train=False)
            logits = eng.forward(m.flat, [inputs_x, inputs_u_s], train=not frozen)
        dl = self._dlogits
        call("es_poly_ce_fwd_bwd", ptr(logits), C, ptr(targets_x), ptr(self.class_weights), B, C, 2.0, 1.0 / B,
             ptr(dl), C, ptr(stats[0:1]), s)
        lam = float(cfg.TRAIN.LAMBDA_U)
        call("es_fm_consistency_fwd_bwd", ptr(logits_w), C, ptr(logits[B:]), C, nu, C, float(cfg.TRAIN.THRES),
             lam / nu, ptr(self._pl), ptr(self._mask), None, ptr(dl[B:]), C, ptr(stats[1:3]), s)
        torch.add(stats[0], stats[1], alpha=lam, out=stats[3])
        if frozen:
            eng.head_backward(m.flat, m.flat_grad, dl, train=False)
            return stats, None
        gb = dist.GradBuckets(m.flat_grad) if dist.world_size() > 1 and self.overlap_allreduce else None
        eng.backward(m.flat, m.flat_grad, dl, grad_ready=gb.ready if gb is not None else None)
        return stats, gb

    def _graphable(self):
        eng = self.model.engine()
        return (self.use_graph and eng.probe is None and not (dist.world_size() > 1 and self.overlap_allreduce))

    def static_batch(self):
        """The captured graph's input buffers as a batch (fill them in place to skip the copy)."""
        if getattr(self, "_graph", None) is None:
            return None
        x, y, uw, us = self._gin
        return ((x, y), ((uw, us), None))

    def _run_graph(self, inputs):
        key = tuple((tuple(t.shape), t.dtype) for t in inputs)
        if getattr(self, "_graph", None) is None or self._gkey != key:
            self._graph = None
            stats, _ = self._compute(*inputs)  # eager step (warms every launch path on this shape)
            gin = [t.clone() for t in inputs]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                gstats, _ = self._compute(*gin)
            self._graph, self._gkey, self._gin, self._gstats = g, key, gin, gstats
            return stats
        for dst, src in zip(self._gin, inputs):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        self._graph.replay()
        return self._gstats

    def step(self, batch):
        """batch = ((x, y), ((u_w, u_s), idx)) -> dict of device scalars / tensors."""
        (inputs_x, targets_x), ((inputs_u_w, inputs_u_s), _) = batch
        dev = self.model.flat.device
        self._inflight.wait()
        inputs = (inputs_x.to(dev, non_blocking=True), targets_x.to(dev, non_blocking=True).to(torch.int64),
                  inputs_u_w.to(dev, non_blocking=True), inputs_u_s.to(dev, non_blocking=True))
        m = self.model
        eng = m.engine()
        eng.pack(m.flat, m.version)
        gb = None
        if self._graphable():
            stats = self._run_graph(inputs)
        else:
            stats, gb = self._compute(*inputs)
        gscale = gb.finish() if gb is not None else dist.allreduce_sum_(m.flat_grad)
        ema = self.ema_model
        self.optimizer.step(ema_flat=ema.ema.flat if ema is not None else None,
                            ema_decay=float(ema.decay) if ema is not None else 0.0, grad_scale=gscale)
        if ema is not None:
            ema.ema.mark_updated()
        self._inflight.record()
        return {"loss": stats[3], "lx": stats[0], "lu": stats[1], "mask_mean": stats[2],
                "pseudo_label": self._pl, "mask": self._mask}

    def train_one(self, epoch):
        self.model.train()
        labeled_iter = iter(self.train_labeled_dl)
        unlabeled_iter = iter(self.train_unlabeled_dl)
        summary_loss = AverageMeter()
        pending = []
        for batch_idx in range(self.config.TRAIN.EVAL_STEP):
            try:
                lab = _next(labeled_iter)
            except StopIteration:
                labeled_iter = iter(self.train_labeled_dl)
                lab = _next(labeled_iter)
            try:
                unl = _next(unlabeled_iter)
            except StopIteration:
                unlabeled_iter = iter(self.train_unlabeled_dl)
                unl = _next(unlabeled_iter)
            out = self.step((lab, unl))
            if self.lr_scheduler is not None:
                self.lr_scheduler.step_update(epoch * self.config.TRAIN.EVAL_STEP + batch_idx)
            pending.append(out["loss"].detach().clone())
        for v in pending:  # one host sync per epoch instead of one per step (code/fixmatch.py:130)
            summary_loss.update(v.item(), self.config.DATA.BATCH_SIZE)
        return summary_loss

    def evaluate_one(self, show_metric=False, show_report=False, show_cf_matrix=False):
        eval_model = self.ema_model.ema if self.config.TRAIN.USE_EMA else self.model
        eval_model.eval()
        summary_loss = AverageMeter()
        outs, tgts = [], []
        with torch.no_grad():
            for images, targets in self.valid_dl:
                images = images.to(self.model.flat.device, non_blocking=True)
                targets = targets.to(self.model.flat.device, non_blocking=True)
                outputs = eval_model(images)
                losses = ce_loss(outputs, targets, reduction='mean')
                summary_loss.update(losses.item(), self.config.DATA.BATCH_SIZE)
                outs.append(outputs.argmax(1).cpu().numpy())
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
        """Same dict keys and filename scheme as code/fixmatch.py:181-202."""
        checkpoint = {}
        if self.config.TRAIN.USE_EMA:
            checkpoint['ema_state_dict'] = self.ema_model.ema.state_dict()
        d = date.today().strftime("%m_%d_%Y")
        h = datetime.now().strftime("%H_%M_%S").split('_')
        h[0] = str(int(h[0]) + 2)
        filename = d + '_' + '_'.join(h) + '_epoch_' + str(self.epoch) + '_size_' + str(self.config.DATA.IMG_SIZE)
        checkpoint['epoch'] = self.epoch
        checkpoint['best_valid_perf'] = self.best_valid_perf
        checkpoint['model_state_dict'] = self.model.state_dict()
        checkpoint['optimizer'] = self.optimizer.state_dict()
        checkpoint['scheduler'] = self.lr_scheduler.state_dict() if self.lr_scheduler is not None else {}
        f = os.path.join(foldname, filename + '.pth')
        torch.save(checkpoint, f)
        print('Saved checkpoint')
        return f

    def load_checkpoint(self, checkpoint_dir, is_train=False):
        checkpoint = torch.load(checkpoint_dir, map_location='cpu', weights_only=True)
        self.model.load_state_dict(checkpoint['model_state_dict'])
        # code/fixmatch.py:204-216: is_train -> trainable again (the IS_FREEZE split re-applied), else frozen
        for p in self.model.parameters():
            p.requires_grad = bool(is_train) and not getattr(self, "frozen", False)
        if is_train and getattr(self, "frozen", False):
            for mod in self._trainable_when_frozen():
                mod.requires_grad_(True)
        if self.config.TRAIN.USE_EMA:
            self.ema_model.ema.load_state_dict(checkpoint['ema_state_dict'])
        self.epoch_start = checkpoint['epoch']
        self.best_valid_perf = checkpoint['best_valid_perf']
        self.optimizer.load_state_dict(checkpoint['optimizer'])
        if self.lr_scheduler is not None:
            self.lr_scheduler.load_state_dict(checkpoint['scheduler'])

    def fit(self):
        if self.epoch_start == self.config.TRAIN.EPOCHS:
            valid_loss, valid_metric = self.evaluate_one()
            print(f'\tValid Loss: {valid_loss.avg:.3f}')
            print(f'\tMetric: {valid_metric}')
            return
        for epoch in range(self.epoch_start, self.config.TRAIN.EPOCHS + 1):
            self.epoch = epoch
            lr = self.optimizer.param_groups[0]["lr"]
            best = f"{float(self.best_valid_perf):.3f}" if self.best_valid_perf else "inf"
            print(f'Training epoch: {self.epoch} | Current LR: {lr:.6f} | The best loss: {best}')
            train_loss = self.train_one(self.epoch)
            print(f'\tTrain Loss: {train_loss.avg:.3f}')
            if epoch % self.config.TRAIN.FREQ_EVAL == 0 and self.valid_dl is not None:
                valid_loss, valid_metric = self.evaluate_one()
                if self.best_valid_perf is None or self.best_valid_perf > valid_loss.avg:
                    self.best_valid_perf = valid_loss.avg
                if dist.rank() == 0:
                    self.save_checkpoint(self.config.TRAIN.SAVE_CP)
                print(f'\tValid Loss: {valid_loss.avg:.3f}')
                print(f'\tMetric: {valid_metric}')
