"""CoMatch trainer with the reference's API (code/comatch.py:18-351) over the native step.

Same constructor and methods as the reference (get_dataloader, get_config, train_one,
evaluate_one, save_checkpoint, load_checkpoint, fit) plus `step(batch)`.  One step
(code/comatch.py:141-231):

  fwd    (logits, fts, z) = model([x; u_w; u_s0; u_s1])   one trunk pass over B + 3 muB images,
                                                         ModelwEmb heads (BatchNorm1d couples rows)
  loss   L_x = PolyCE(logits_x, y, w)                             (:156-160)
         pseudo-labels: softmax(l_w) -> DA (<= 32 batch means) -> memory smoothing against the
         bank -> max / mask (>= THRES)                            (:162-185)
         gated bank write (only when B + muB == queue_size)       (:187-196)
         L_c = contrastive(z_s0, z_s1 | Q = p p^T graph)          (:199-213)
         L_u = focal(logits_s0 | p, mask)                         (:215-220)
         losses = L_x + LAMBDA_U L_u + LAMBDA_C L_c               (:222)
  bwd    heads backward -> dL/dfts -> trunk backward over every image (BN1d couples the rows)
  comm   data-parallel only (global-batch semantics: N ranks compute what one process computes on
         the concatenated batch): all-reduce of the DA batch mean (C floats); all-gather of the bank
         rows (every rank holds the same bank); SyncBatchNorm1d in the head (all-reduced per-feature
         sums, comatch_model.EmbHeads); the contrastive graph over the global batch (all-gathered
         z_s1 / probs columns, summed column gradients); RCCL all-reduce of the flat grad
  opt    Adam + parameter EMA in one sweep, EMA of the BatchNorm buffers, lr_scheduler.step_update

Reference behaviour kept on purpose: `train_one` walks the whole unlabeled
loader, and the labeled batch comes from a FRESH iterator every step (`next()` on the DataLoader
raises, code/comatch.py:135-138), i.e. always its first batch.
"""
import numpy as np
import torch

from . import _lib, dist
from ._lib import call, ptr
from .fixmatch import FixMatch, _next
from .loss import ce_loss
from .utils import AverageMeter, calculate_metrics

HIST_CAP = 32  # distribution-alignment history (code/comatch.py:169-170)


class CoMatch(FixMatch):
    def __init__(self, model, opt_func="Adam", lr=1e-3, device='cpu'):
        super().__init__(model, opt_func=opt_func, lr=lr, device=device)
        # code/comatch.py:29-39
        self.queue_batch = 5
        self.alpha = 0.9
        self.temperature = 0.2
        self.contrast_th = 0.8
        self.gamma = 2
        self._ws = {}

    def _trainable_when_frozen(self):
        """code/comatch.py:64-73: `model.fc` and `model.head_emb`."""
        return [self.model.fc, self.model.head_emb]

    def get_config(self, config):
        super().get_config(config)
        dev = self.model.flat.device
        self.low_dim = config.MODEL.LOW_DIM
        if self.low_dim != self.model.cfg.low_dim:
            raise ValueError(f"MODEL.LOW_DIM={self.low_dim} but the model was built with {self.model.cfg.low_dim}")
        C = config.MODEL.NUM_CLASSES
        # code/comatch.py:90-96
        self.queue_size = self.queue_batch * (config.DATA.MU + 1) * config.DATA.BATCH_SIZE
        self.queue_feats = torch.zeros(self.queue_size, self.low_dim, device=dev)
        self.queue_probs = torch.zeros(self.queue_size, C, device=dev)
        self.queue_ptr = 0
        self.prob_hist = torch.zeros(HIST_CAP, C, device=dev)
        self._hist_len, self._hist_pos = 0, -1

    def set_queue_size(self, q):
        """Resize (and clear) the memory bank -- e.g. the 65,536-entry bank of BASELINE config C1;
        the reference derives it from queue_batch (code/comatch.py:91)."""
        dev = self.model.flat.device
        self.queue_size = int(q)
        self.queue_feats = torch.zeros(self.queue_size, self.low_dim, device=dev)
        self.queue_probs = torch.zeros(self.queue_size, self.queue_probs.shape[1], device=dev)
        self.queue_ptr = 0
        self._ws = {}  # the pseudo-label workspace is sized by the queue size

    @property
    def prob_list(self):
        """The DA history as the reference's list of per-batch mean probabilities, oldest first."""
        idx = [(self._hist_pos - self._hist_len + 1 + j) % HIST_CAP for j in range(self._hist_len)]
        return [self.prob_hist[i] for i in idx]

    def _workspace(self, bt, btu, C, L):
        key = (bt, btu, self.queue_size)
        if key not in self._ws:
            dev = self.model.flat.device
            n = bt + 3 * btu
            lib = _lib.load()
            self._ws[key] = {
                "dl": torch.zeros(n, C, device=dev), "dz": torch.zeros(n, L, device=dev),
                "probs": torch.zeros(btu, C, device=dev), "probs_orig": torch.zeros(btu, C, device=dev),
                "pl": torch.zeros(btu, dtype=torch.int32, device=dev), "mask": torch.zeros(btu, device=dev),
                "ws_p": torch.zeros(lib.es_comatch_pseudo_workspace(btu, C, self.queue_size), device=dev),
                "ws_c": torch.zeros(lib.es_comatch_contrastive_workspace(btu), device=dev),
                "ws_f": torch.zeros(btu, device=dev)}
        return self._ws[key]

    # ------------------------------------------------------------------ the hot step
    def step(self, batch, drop_keep=None):
        """batch = ((x, y), ((u_w, u_s0, u_s1), idx)) -> dict of device scalars / tensors.
        drop_keep: optional uint8 [B + 3muB, D/4] Dropout keep-mask to replay (parity tests)."""
        (inputs_x, targets_x), ((u_w, u_s0, u_s1), _) = batch
        dev = self.model.flat.device
        self._inflight.wait()
        inputs_x = inputs_x.to(dev, non_blocking=True)
        targets_x = targets_x.to(dev, non_blocking=True).to(torch.int64)
        u_w, u_s0, u_s1 = (t.to(dev, non_blocking=True) for t in (u_w, u_s0, u_s1))
        cfg, m = self.config, self.model
        bt, btu = int(inputs_x.shape[0]), int(u_w.shape[0])
        C, L = m.cfg.num_classes, m.cfg.low_dim
        s = _lib.stream()
        W = self._workspace(bt, btu, C, L)
        keep = None if drop_keep is None else drop_keep.to(dev, torch.uint8).contiguous()
        frozen = getattr(self, "frozen", False)  # IS_FREEZE: the trunk in inference form, heads trained
        logits, fts, z = m._run([inputs_x, u_w, u_s0, u_s1], train=True, keep=keep, trunk_train=not frozen)
        lw, ls0 = logits[bt:bt + btu], logits[bt + btu:bt + 2 * btu]
        zx, zw, z0, z1 = z[:bt], z[bt:bt + btu], z[bt + btu:bt + 2 * btu], z[bt + 2 * btu:]
        dl, dz = W["dl"], W["dz"]
        stats = torch.empty(5, dtype=torch.float32, device=dev)  # lx, lu, lc, mask_mean, total
        lam_u, lam_c = float(cfg.TRAIN.LAMBDA_U), float(cfg.TRAIN.LAMBDA_C)

        call("es_poly_ce_fwd_bwd", ptr(logits), C, ptr(targets_x), ptr(self.class_weights), bt, C, 2.0, 1.0 / bt,
             ptr(dl), C, ptr(stats[0:1]), s)
        self._hist_pos = (self._hist_pos + 1) % HIST_CAP
        self._hist_len = min(self._hist_len + 1, HIST_CAP)
        world = dist.world_size()
        hist_given = 0
        if world > 1:  # DA over the global batch: the ranks' batch means, averaged (equal shards)
            row = self.prob_hist[self._hist_pos]
            call("es_softmax_colmean", ptr(lw), C, btu, C, ptr(row), s)
            dist.allreduce_mean_(row)
            hist_given = 1
        call("es_comatch_pseudo_ex", ptr(lw), C, btu, C, ptr(self.prob_hist), HIST_CAP, self._hist_len,
             self._hist_pos, hist_given, ptr(zw), L, L, ptr(self.queue_feats), ptr(self.queue_probs),
             self.queue_size, self.temperature, self.alpha, float(cfg.TRAIN.THRES), ptr(W["probs"]),
             ptr(W["probs_orig"]), ptr(W["pl"]), ptr(W["mask"]), ptr(W["ws_p"]), s)
        n = world * (bt + btu)  # code/comatch.py:192: the (global) batch against the queue size
        if n == self.queue_size:  # code/comatch.py:192-196
            if world == 1:
                call("es_comatch_bank_write", ptr(zw), L, btu, ptr(zx), L, bt, L, ptr(W["probs_orig"]),
                     ptr(targets_x), C, ptr(self.queue_feats), ptr(self.queue_probs), self.queue_ptr,
                     self.queue_size, s)
            else:  # every rank writes every rank's rows, in rank order: identical banks
                zw_a, zx_a = dist.all_gather_cat(zw.contiguous()), dist.all_gather_cat(zx.contiguous())
                po_a, y_a = dist.all_gather_cat(W["probs_orig"]), dist.all_gather_cat(targets_x)
                for r in range(world):
                    call("es_comatch_bank_write", ptr(zw_a[r * btu:]), L, btu, ptr(zx_a[r * bt:]), L, bt, L,
                         ptr(po_a[r * btu:]), ptr(y_a[r * bt:]), C, ptr(self.queue_feats), ptr(self.queue_probs),
                         self.queue_ptr + r * (bt + btu), self.queue_size, s)
            self.queue_ptr = (self.queue_ptr + n) % self.queue_size
        if world == 1:
            call("es_comatch_contrastive_fwd_bwd", ptr(z0), L, ptr(z1), L, ptr(W["probs"]), btu, L, C,
                 self.temperature, self.contrast_th, lam_c / btu, ptr(stats[2:3]), ptr(dz[bt + btu:]), L,
                 ptr(dz[bt + 2 * btu:]), L, ptr(W["ws_c"]), s)
        else:
            # the graph spans the global batch (code/comatch.py:200-213 on the concatenated batch): this
            # rank's anchor rows against every rank's z_s1 / probs columns (all-gathered, rank order =
            # global order, so the self-loop sits at column rank * btu + i).  Gradient scale lam_c / btu =
            # lam_c * world / nu_global: the flat gradient is SUM-reduced and scaled by 1 / world.  Every
            # rank holds a share of d/dz_s1 for all columns; the shares are summed and each keeps its rows.
            rk, nc = dist.rank(), world * btu
            z1_all = dist.all_gather_cat(z1.contiguous())
            p_all = dist.all_gather_cat(W["probs"])
            if "ws_cx" not in W or W["ws_cx"].numel() < _lib.load().es_comatch_contrastive_ex_workspace(btu, nc):
                W["ws_cx"] = torch.zeros(_lib.load().es_comatch_contrastive_ex_workspace(btu, nc), device=dev)
                W["dz1_all"] = torch.zeros(nc, L, device=dev)
            call("es_comatch_contrastive_fwd_bwd_ex", ptr(z0), L, ptr(z1_all), L, ptr(W["probs"]), ptr(p_all), btu, nc,
                 rk * btu, L, C, self.temperature, self.contrast_th, lam_c / btu, float(nc), ptr(stats[2:3]),
                 ptr(dz[bt + btu:]), L, ptr(W["dz1_all"]), L, ptr(W["ws_cx"]), s)
            dist.allreduce_inplace_(W["dz1_all"])
            dz[bt + 2 * btu:].copy_(W["dz1_all"][rk * btu:(rk + 1) * btu])
            dist.allreduce_inplace_(stats[2:3])  # L_c over the global batch (each rank sent its rows' sum / nc)
        call("es_comatch_focal_fwd_bwd", ptr(ls0), C, ptr(W["probs"]), ptr(W["mask"]), btu, C, float(self.gamma),
             lam_u / btu, ptr(stats[1:2]), ptr(dl[bt + btu:]), C, ptr(W["ws_f"]), s)
        torch.mean(W["mask"], 0, keepdim=True, out=stats[3:4])
        torch.add(stats[0], stats[1], alpha=lam_u, out=stats[4])
        stats[4].add_(stats[2], alpha=lam_c)

        gb = dist.GradBuckets(m.flat_grad) if world > 1 and self.overlap_allreduce else None
        m.backward_from(dl, dz, grad_ready=gb.ready if gb is not None else None, trunk=not frozen)
        gscale = gb.finish() if gb is not None else dist.allreduce_sum_(m.flat_grad)
        ema = self.ema_model
        self.optimizer.step(ema_flat=ema.ema.flat if ema is not None else None,
                            ema_decay=float(ema.decay) if ema is not None else 0.0, grad_scale=gscale)
        if ema is not None:
            ema.update_buffers(m)
            ema.ema.mark_updated()
        self._inflight.record()
        return {"loss": stats[4], "lx": stats[0], "lu": stats[1], "lc": stats[2], "mask_mean": stats[3],
                "pseudo_label": W["pl"], "mask": W["mask"], "probs": W["probs"], "probs_orig": W["probs_orig"],
                "logits": logits, "fts": fts, "z": z}

    def train_one(self, epoch):
        """Whole unlabeled loader per epoch; the labeled batch from a fresh iterator each step, as
        the reference (code/comatch.py:131-138)."""
        self.model.train()
        summary_loss = AverageMeter()
        pending = []
        for batch_idx, unl in enumerate(self.train_unlabeled_dl):
            lab = _next(iter(self.train_labeled_dl))
            out = self.step((lab, unl))
            if self.lr_scheduler is not None:
                self.lr_scheduler.step_update(epoch * self.config.TRAIN.EVAL_STEP + batch_idx)
            pending.append(out["loss"].detach().clone())
        for v in pending:
            summary_loss.update(v.item(), self.config.DATA.BATCH_SIZE)
        return summary_loss

    def evaluate_one(self, show_metric=False, show_report=False, show_cf_matrix=False):
        """code/comatch.py:237-281: EMA (or live) model in eval mode, `outputs, _, _ = model(x)`."""
        eval_model = self.ema_model.ema if self.config.TRAIN.USE_EMA else self.model
        eval_model.eval()
        summary_loss = AverageMeter()
        outs, tgts = [], []
        with torch.no_grad():
            for images, targets in self.valid_dl:
                images = images.to(self.model.flat.device, non_blocking=True)
                targets = targets.to(self.model.flat.device, non_blocking=True)
                outputs, _, _ = eval_model(images)
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
