"""Loss surface of code/loss.py, computed by the fused HIP kernels (losses.hip).

`ce_loss` / `consistency_loss` keep the reference signatures (code/loss.py:90,126) and return
autograd-capable tensors: each kernel computes the value AND d(value)/d(logits) in one launch,
the backward just scales the saved gradient.  Only the branches the SSL path uses are native
(poly / plain hard-label CE, hard-label 'ce' consistency); the others (focal, LDAM, soft labels,
margin losses, 'L2') are outside the hot path and raise.
"""
import torch

from . import _lib
from ._lib import call, ptr


class _CE(torch.autograd.Function):
    """PolyLoss(softmax=True, epsilon) mean (code/loss.py:308-364); epsilon=0 -> plain CE mean."""

    @staticmethod
    def forward(ctx, logits, targets, weights, epsilon):
        lg = logits.detach().float().contiguous()
        n, C = lg.shape
        tg = targets.to(torch.int64).contiguous()
        out = torch.empty(1, dtype=torch.float32, device=lg.device)
        dl = torch.empty_like(lg)
        w = None if weights is None else weights.float().contiguous()
        call("es_poly_ce_fwd_bwd", ptr(lg), C, ptr(tg), ptr(w), n, C, float(epsilon), 1.0 / n, ptr(dl), C, ptr(out),
             _lib.stream())
        ctx.save_for_backward(dl)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None, None, None


class _Consistency(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits_w, logits_s, tau):
        lw = logits_w.detach().float().contiguous()
        ls = logits_s.detach().float().contiguous()
        n, C = ls.shape
        out = torch.empty(2, dtype=torch.float32, device=ls.device)
        dls = torch.empty_like(ls)
        pl = torch.empty(n, dtype=torch.int32, device=ls.device)
        mask = torch.empty(n, dtype=torch.uint8, device=ls.device)
        call("es_fm_consistency_fwd_bwd", ptr(lw), C, ptr(ls), C, n, C, float(tau), 1.0 / n, ptr(pl), ptr(mask), None,
             ptr(dls), C, ptr(out), _lib.stream())
        ctx.save_for_backward(dls)
        ctx.mark_non_differentiable(out)
        return out[0], out[1], pl, mask

    @staticmethod
    def backward(ctx, g_loss, g_mask, g_pl, g_m):
        (dls,) = ctx.saved_tensors
        return None, dls * g_loss, None


def ce_loss(logits, targets, class_weights=None, use_hard_labels=True, reduction='none', type_loss='none',
            cls_num_list=None):
    """code/loss.py:90-124.  Native: type_loss='poly' (mean) and plain hard-label CE (mean, unweighted)."""
    if not use_hard_labels:
        raise NotImplementedError("soft-label ce_loss is not on the SSL hot path (code/loss.py:120-124)")
    if type_loss == 'poly':
        if reduction != 'mean':
            raise NotImplementedError("native PolyLoss implements reduction='mean' (the trainers' only use)")
        return _CE.apply(logits, targets, class_weights, 2.0)
    if type_loss in ('focal', 'ldam'):
        raise NotImplementedError(f"type_loss={type_loss!r} is outside the SSL hot path (SURVEY.md §2 row 4)")
    if reduction == 'mean' and class_weights is None:
        return _CE.apply(logits, targets, None, 0.0)
    raise NotImplementedError("plain CE: native path implements reduction='mean' without class weights")


def consistency_loss(logits_w, logits_s, name='ce', T=1.0, p_cutoff=0.0, use_hard_labels=True, device=None,
                     loss_fc=None, fc=None):
    """code/loss.py:126-164 -> (masked CE mean, mask mean).  `T` is unused on the hard-label path
    (reference quirk)."""
    if loss_fc is not None and fc is not None:
        raise NotImplementedError("margin-loss consistency (code/loss.py:133-141) is not on the SSL path")
    if name != 'ce' or not use_hard_labels:
        raise NotImplementedError("native consistency_loss implements name='ce', use_hard_labels=True")
    loss, mask_mean, _, _ = _Consistency.apply(logits_w, logits_s, p_cutoff)
    return loss, mask_mean


def consistency_loss_full(logits_w, logits_s, p_cutoff):
    """Same as consistency_loss, also returning int32 pseudo-labels and the uint8 mask."""
    return _Consistency.apply(logits_w, logits_s, p_cutoff)


def weighted_ce_fwd_bwd(logits, targets, weights, dlogits, out):
    """F.cross_entropy(logits, y, weight=w, reduction='mean') = sum_i w[y_i] l_i / sum_i w[y_i]
    (code/loss.py:118: the supervised step, code/supervised.py:127-130, and the SemiFormer heads,
    code/semiformer.py:125-126): out[0] and dlogits = d(out[0])/d(logits) in one launch.

    Data-parallel (world > 1) with class weights, the rows are this rank's shard of the global batch:
    the denominator is the weight sum over EVERY rank's rows (es_ce_weight_sum + one SUM all-reduce of
    a float, no host sync), so the rank writes its share sum_{own} w l / W_global and the gradient of
    that share times `world`; the optimizer's SUM all-reduce of the flat gradient times 1/world then
    yields d(global weighted mean) -- what the single-process reference computes over the whole batch.
    A per-rank weighted mean would instead average sum_r W_r-normalised means, which differs whenever
    the shards' weight sums differ.  out[0] is all-reduced too, so every rank logs the global loss.
    Without weights the shards are equal-sized plain means and the DDP average is already exact."""
    from . import dist
    n, C = logits.shape
    world = dist.world_size()
    if weights is None or world == 1:
        call("es_ce_weighted_fwd_bwd", ptr(logits), C, ptr(targets), ptr(weights), n, C, 1.0, ptr(dlogits), C, ptr(out),
             _lib.stream())
        return
    wsum = torch.empty(1, dtype=torch.float32, device=logits.device)
    call("es_ce_weight_sum", ptr(targets), ptr(weights), n, C, ptr(wsum), _lib.stream())
    dist.allreduce_inplace_(wsum)
    call("es_ce_weighted_fwd_bwd_global", ptr(logits), C, ptr(targets), ptr(weights), ptr(wsum), n, C, float(world),
         ptr(dlogits), C, ptr(out), _lib.stream())
    dist.allreduce_inplace_(out[:1])
