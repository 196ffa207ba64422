"""Bound on how many training steps the host queues ahead of the GPU (all trainers)."""
import os

import torch

# How many steps the host may queue ahead of the GPU.  The conv weight-gradient side stream and the
# branch streams record_stream() their operands, so the caching allocator can recycle a step's
# activations only once the GPU has passed that step's events: a host queueing step i+1 while the
# GPU still runs step i's backward allocates step i+1's maps fresh, and at Conformer-B/384 sizes
# (~85 GB allocated per step) the reserved pool then reaches the whole HBM, where each allocation
# retry flushes the cache and stalls (S1 measured 5x slower).  Depth 1 = the next step starts its
# host work once the previous step's last kernel (the Adam + EMA sweep) has finished (the Conformer
# / ResNet trainers); 2 for the ViT trainers, whose engine keeps its activations in its own
# buffers (F1: 35.1 ms at depth 2 and unbounded, 35.5 ms at depth 1).  ENDOSSL_MAX_INFLIGHT_STEPS
# overrides both; 0 = unbounded.
_ENV_DEPTH = os.environ.get("ENDOSSL_MAX_INFLIGHT_STEPS")


class StepThrottle:
    """Bounds a trainer's queued steps to `depth` (record() after a step's last launch, wait() before
    the next step's first)."""

    def __init__(self, depth=1):
        self.depth = int(_ENV_DEPTH) if _ENV_DEPTH is not None else depth
        self.events = []

    def record(self):
        if self.depth <= 0 or not torch.cuda.is_available():
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.events.append(ev)

    def wait(self):
        while self.depth > 0 and len(self.events) >= self.depth:
            self.events.pop(0).synchronize()
