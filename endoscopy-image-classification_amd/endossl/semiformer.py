"""SemiFormer trainer with the reference's API (code/semiformer.py:18-262) over the native Conformer.

Same constructor and methods -- get_dataloader, get_config, train_one, evaluate_one,
save_checkpoint, load_checkpoint, fit -- plus `step(batch)` (one SSL step) and `step_sup(batch)`
(the supervised warm-up step of epochs < TRAIN.EVAL_STEP_SUP).  One SSL step (:103-146):

  fwd    (out_conv, out_trans) = model([x; u_w; u_s])   one pass over B + 2muB images: BatchNorm
                                                         couples the rows, so every row is kept
  loss   lx = CE_w(out_conv[:B], y) + CE_w(out_trans[:B], y)          fused value+grad kernels
         lu = consistency(conv weak, conv strong) + consistency(conv weak, trans strong)
              -- the CONV head's weak logits supervise both heads
         losses = lx + LAMBDA_U * lu
  bwd    autograd over the HIP ops from d(losses)/d(logits) (weak rows: zero, detached)
  opt    Adam + EMA of the parameters in one sweep, EMA of the BatchNorm buffers, LR update
"""
import os
from datetime import date, datetime

import numpy as np
import torch

from . import _lib, dist
from .conformer import join_wgrad_stream
from ._lib import call, ptr
from .ema import ModelEMA
from .fixmatch import _next
from .loss import weighted_ce_fwd_bwd
from .lr_scheduler import build_scheduler
from .optimizer import build_optimizer
from .throttle import StepThrottle
from .utils import AverageMeter, balanced_class_weights, calculate_metrics


class SemiFormer:
    def __init__(self, model, opt_func="Adam", lr=1e-3, device='cpu'):
        self.model = model
        self.opt_func = opt_func
        self.device = device
        self.model.to(self.device)
        self.epoch_start = 0
        self.best_valid_perf = None
        self._inflight = StepThrottle()

    def get_dataloader(self, train_dl, valid_dl, test_dl=None):
        self.train_labeled_dl, self.train_unlabeled_dl = train_dl
        self.valid_dl = valid_dl
        self.test_dl = test_dl

    def get_config(self, config):
        self.config = config
        print('Training mode: SemiFormer')
        dist.broadcast_(self.model.flat)
        self.model.mark_updated()
        self.ema_model = ModelEMA(model=self.model, decay=config.TRAIN.EMA_DECAY, device=self.device) \
            if config.TRAIN.USE_EMA else None
        # code/semiformer.py:50-56: IS_FREEZE trains conv_cls_head and trans_cls_head only; the native
        # forward then keeps the trunk off the autograd tape (NativeConformer.frozen_trunk) so only the
        # heads' backward runs, and the trunk's gradient stays exactly zero
        self.frozen = bool(config.TRAIN.IS_FREEZE)
        self.model.frozen_trunk = self.frozen
        if self.frozen:
            for p in self.model.parameters():
                p.requires_grad = False
            self.model.conv_cls_head.requires_grad_(True)
            self.model.trans_cls_head.requires_grad_(True)
        self.optimizer = build_optimizer(self.model, opt_func=self.opt_func, lr=config.TRAIN.BASE_LR)
        self.lr_scheduler = build_scheduler(config=config, optimizer=self.optimizer,
                                            n_iter_per_epoch=config.TRAIN.EVAL_STEP)
        if config.TRAIN.CLS_WEIGHT:
            df = self.train_labeled_dl.dataset.df
            self.class_weights = torch.tensor(balanced_class_weights(df[config.DATA.TARGET_NAME]),
                                              dtype=torch.float).to(self.device)
        else:
            self.class_weights = None

    # ------------------------------------------------------------------ steps
    def _ce(self, logits, y, dl, out):
        weighted_ce_fwd_bwd(logits, y, self.class_weights, dl, out)

    def _finish(self, out_conv, out_trans, dconv, dtrans):
        self.optimizer.zero_grad()
        torch.autograd.backward([out_conv, out_trans], [dconv, dtrans])
        join_wgrad_stream(self.model.flat.device)  # (the backward's final callback already did)
        gscale = dist.allreduce_sum_(self.model.flat_grad)
        ema = self.ema_model
        self.optimizer.step(ema_flat=ema.ema.flat if ema is not None else None,
                            ema_decay=float(ema.decay) if ema is not None else 0.0, grad_scale=gscale)
        if ema is not None:
            ema.update_buffers(self.model)
            ema.ema.mark_updated()
        self._inflight.record()

    def step(self, batch):
        """batch = ((x, y), ((u_w, u_s), idx)) -> dict of device scalars / tensors."""
        (inputs_x, targets_x), ((inputs_u_w, inputs_u_s), _) = batch
        dev = self.model.flat.device
        self._inflight.wait()
        bs, nu = int(inputs_x.shape[0]), int(inputs_u_w.shape[0])
        targets_x = targets_x.to(dev, non_blocking=True).to(torch.int64).contiguous()
        inputs = torch.cat((inputs_x.to(dev), inputs_u_w.to(dev), inputs_u_s.to(dev)))
        self.model.train()
        out_conv, out_trans = self.model(inputs)
        C = out_conv.shape[1]
        lam = float(self.config.TRAIN.LAMBDA_U)
        s = _lib.stream()
        stats = torch.zeros(7, dtype=torch.float32, device=dev)  # lx_c, lx_t, lu_c, mask, lu_t, mask, total
        pl = torch.empty(nu, dtype=torch.int32, device=dev)
        mask = torch.empty(nu, dtype=torch.uint8, device=dev)
        dconv = torch.zeros_like(out_conv)
        dtrans = torch.zeros_like(out_trans)
        oc, ot = out_conv.detach(), out_trans.detach()
        self._ce(oc[:bs], targets_x, dconv[:bs], stats[0:1])
        self._ce(ot[:bs], targets_x, dtrans[:bs], stats[1:2])
        weak = oc[bs:bs + nu]
        call("es_fm_consistency_fwd_bwd", ptr(weak), C, ptr(oc[bs + nu:]), C, nu, C, float(self.config.TRAIN.THRES),
             lam / nu, ptr(pl), ptr(mask), None, ptr(dconv[bs + nu:]), C, ptr(stats[2:4]), s)
        call("es_fm_consistency_fwd_bwd", ptr(weak), C, ptr(ot[bs + nu:]), C, nu, C, float(self.config.TRAIN.THRES),
             lam / nu, None, None, None, ptr(dtrans[bs + nu:]), C, ptr(stats[4:6]), s)
        lx = stats[0] + stats[1]
        lu = stats[2] + stats[4]
        loss = lx + lam * lu
        self._finish(out_conv, out_trans, dconv, dtrans)
        return {"loss": loss, "lx": lx, "lu": lu, "mask_mean": stats[5], "pseudo_label": pl, "mask": mask,
                "out_conv": oc, "out_trans": ot}

    def step_sup(self, batch):
        """Supervised warm-up step (code/semiformer.py:75-101): CE on both heads."""
        images, targets = batch
        dev = self.model.flat.device
        self._inflight.wait()
        targets = targets.to(dev).to(torch.int64).contiguous()
        self.model.train()
        out_conv, out_trans = self.model(images.to(dev))
        stats = torch.zeros(2, dtype=torch.float32, device=dev)
        dconv, dtrans = torch.zeros_like(out_conv), torch.zeros_like(out_trans)
        self._ce(out_conv.detach(), targets, dconv, stats[0:1])
        self._ce(out_trans.detach(), targets, dtrans, stats[1:2])
        self._finish(out_conv, out_trans, dconv, dtrans)
        return {"loss": stats.sum()}

    def train_one(self, epoch):
        self.model.train()
        summary_loss = AverageMeter()
        pending = []
        if epoch < self.config.TRAIN.EVAL_STEP_SUP:
            num_steps = len(self.train_labeled_dl)
            for step, batch in enumerate(self.train_labeled_dl):
                out = self.step_sup(batch)
                self.lr_scheduler.step_update(epoch * num_steps + step)
                pending.append(out["loss"].detach().clone())
        else:
            labeled_iter = iter(self.train_labeled_dl)
            unlabeled_iter = iter(self.train_unlabeled_dl)
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
                self.lr_scheduler.step_update(epoch * self.config.TRAIN.EVAL_STEP + batch_idx)
                pending.append(out["loss"].detach().clone())
        for v in pending:  # one host sync per epoch
            summary_loss.update(v.item(), self.config.DATA.BATCH_SIZE)
        return summary_loss

    def evaluate_one(self, show_metric=False, show_report=False, show_cf_matrix=False):
        """code/semiformer.py:150-198: CE of both heads, prediction = argmax softmax(conv + trans)."""
        eval_model = self.ema_model.ema if self.config.TRAIN.USE_EMA else self.model
        eval_model.eval()
        summary_loss = AverageMeter()
        outs, tgts = [], []
        dev = self.model.flat.device
        with torch.no_grad():
            for images, targets in self.valid_dl:
                out_conv, out_trans = eval_model(images.to(dev))
                targets = targets.to(dev).to(torch.int64).contiguous()
                st = torch.zeros(2, device=dev)
                scratch = torch.empty_like(out_conv)
                call("es_ce_weighted_fwd_bwd", ptr(out_conv), out_conv.shape[1], ptr(targets), None,
                     out_conv.shape[0], out_conv.shape[1], 1.0, ptr(scratch), out_conv.shape[1], ptr(st[0:1]),
                     _lib.stream())
                call("es_ce_weighted_fwd_bwd", ptr(out_trans), out_trans.shape[1], ptr(targets), None,
                     out_trans.shape[0], out_trans.shape[1], 1.0, ptr(scratch), out_trans.shape[1], ptr(st[1:2]),
                     _lib.stream())
                summary_loss.update(st.sum().item(), self.config.DATA.BATCH_SIZE)
                # argmax of softmax(conv + trans) == argmax of (conv + trans)
                outs.append((out_conv + out_trans).argmax(1).cpu().numpy())
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
        """Same dict keys and filename scheme as code/semiformer.py:201-221."""
        checkpoint = {}
        if self.config.TRAIN.USE_EMA:
            checkpoint['ema_state_dict'] = self.ema_model.ema.state_dict()
        d = date.today().strftime("%m_%d_%Y")
        h = datetime.now().strftime("%H_%M_%S").split('_')
        h[0] = str(int(h[0]) + 2)
        filename = d + '_' + '_'.join(h) + '_epoch_' + str(self.epoch)
        checkpoint['epoch'] = self.epoch
        checkpoint['best_valid_perf'] = self.best_valid_perf
        checkpoint['model_state_dict'] = self.model.state_dict()
        checkpoint['optimizer'] = self.optimizer.state_dict()
        checkpoint['scheduler'] = self.lr_scheduler.state_dict()
        f = os.path.join(foldname, filename + '.pth')
        torch.save(checkpoint, f)
        print('Saved checkpoint')
        return f

    def load_checkpoint(self, checkpoint_dir, is_train=False):
        checkpoint = torch.load(checkpoint_dir, map_location='cpu', weights_only=True)
        self.model.load_state_dict(checkpoint['model_state_dict'])
        for p in self.model.parameters():
            p.requires_grad = bool(is_train)
        if self.config.TRAIN.USE_EMA:
            self.ema_model.ema.load_state_dict(checkpoint['ema_state_dict'])
        self.epoch_start = checkpoint['epoch']
        self.best_valid_perf = checkpoint['best_valid_perf']
        self.optimizer.load_state_dict(checkpoint['optimizer'])
        self.lr_scheduler.load_state_dict(checkpoint['scheduler'])

    def fit(self):
        for epoch in range(self.epoch_start, self.config.TRAIN.EPOCHS):
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
