"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL ("nccl" backend on
ROCm) on the GPU box, gloo for the CPU tests.  The reference is single-device; the
only exchange the FixMatch/ViT step needs is the mean of the flat fp32 gradient buffer
(rows are independent, loss terms are per-row means over equal shards).  CoMatch adds two small
exchanges (comatch.py): the distribution-alignment batch mean (all-reduce of C floats) and the
memory-bank rows (all-gather), so every rank holds the same DA history and the same bank."""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise from torchrun's RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* (127.0.0.1).  Returns
    (rank, world, local device index)."""
    share = os.environ.get("ENDOSSL_SHARE_DEVICE") == "1"
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), 0 if share else int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0, gloo over HIP tensors
    # (RCCL refuses two ranks on one device).  Not for measurement.
    backend = os.environ.get("ENDOSSL_DIST_BACKEND") or backend
    if share:
        local = 0
        if backend is None:
            backend = "gloo"
        elif backend == "nccl":
            raise RuntimeError("ENDOSSL_SHARE_DEVICE=1 puts every rank on device 0, which RCCL refuses: "
                               "use the gloo backend for the one-GPU rehearsal")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def broadcast_(t, src=0):
    if world_size() > 1:
        dist.broadcast(t, src)
    return t


def allreduce_sum_(t):
    """In-place SUM all-reduce (RCCL ring over xGMI on the GPU box); returns the 1/world scale."""
    w = world_size()
    if w > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return 1.0 / w


_comm_streams = {}


class GradBuckets:
    """Bucketed SUM all-reduce of the flat fp32 gradient, overlapped with the reverse pass (the
    reference's DDP wrapper does this per 25 MB bucket; here one bucket per transformer block, ~7 MB
    at ViT-S, since each block's parameters are contiguous in the flat layout).  The engine calls
    ready(lo, hi, events) as soon as grad[lo:hi] is final; the all-reduce is issued from a side
    stream that waits on those HIP events, so RCCL runs beside the remaining backward kernels.
    finish() all-reduces every range never handed over (embedding, head, final norm, or all of it
    when the engine took a path without the hook), makes the caller's stream wait for every
    collective, and returns the 1/world scale the optimizer applies.  Each element is summed
    exactly once, so the result is bit-identical to one all-reduce of the whole buffer."""

    def __init__(self, grad):
        self.grad = grad
        self.world = world_size()
        self.works = []
        self.ranges = []

    def ready(self, lo, hi, events=()):
        if self.world == 1 or hi <= lo:
            return
        t = self.grad[lo:hi]
        if t.is_cuda:
            dev = t.device
            st = _comm_streams.get(dev)
            if st is None:
                st = _comm_streams[dev] = torch.cuda.Stream(device=dev)
            for ev in events:
                st.wait_event(ev)
            with torch.cuda.stream(st):
                self.works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True))
        else:
            self.works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True))
        self.ranges.append((lo, hi))

    def finish(self):
        if self.world == 1:
            return 1.0
        pos, n = 0, self.grad.numel()
        for lo, hi in sorted(self.ranges) + [(n, n)]:
            if lo > pos:
                self.works.append(dist.all_reduce(self.grad[pos:lo], op=dist.ReduceOp.SUM, async_op=True))
            pos = max(pos, hi)
        for w in self.works:
            w.wait()
        self.works, self.ranges = [], []
        return 1.0 / self.world


def allreduce_inplace_(t):
    """In-place SUM over ranks (SyncBatchNorm statistics, CoMatch's contrastive column gradients)."""
    if world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def allreduce_mean_(t):
    """In-place mean over ranks (CoMatch's distribution-alignment batch mean)."""
    w = world_size()
    if w > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.mul_(1.0 / w)
    return t


def all_gather_cat(t):
    """[world * n, ...] concatenation of every rank's t in rank order (CoMatch's bank rows)."""
    w = world_size()
    if w == 1:
        return t
    t = t.contiguous()
    if dist.get_backend() == "gloo":  # CPU tests: list form
        parts = [torch.empty_like(t) for _ in range(w)]
        dist.all_gather(parts, t)
        return torch.cat(parts)
    out = torch.empty((w * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t)
    return out


def barrier():
    if world_size() > 1:
        dist.barrier()
