"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL ("nccl" backend on
ROCm) on the GPU box, gloo for the CPU tests.  The reference is single-device; the
only exchange the FixMatch/ViT step needs is the mean of the flat fp32 gradient buffer
(rows are independent, loss terms are per-row means over equal shards)."""
import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise from torchrun's RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* (127.0.0.1)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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


def barrier():
    if world_size() > 1:
        dist.barrier()
