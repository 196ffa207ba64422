"""ModelEMA (code/ema.py:40-62): deepcopy + eval, then e <- d*e + (1-d)*m over EVERY state_dict
entry (parameters and buffers; integer buffers blended in fp32 and truncated, as the reference's
`copy_` does).  The update is one launch of es_ema_update_multi over a cached (entry, chunk) table,
instead of the reference's 4 tiny kernels per tensor.  The FixMatch trainer fuses this update into
the Adam sweep instead (es_adam_ema_step) when both models are NativeViT.
"""
import ctypes
from copy import deepcopy

import torch

from . import _lib
from ._lib import call, ptr

_CHUNK = 4096


class ModelEMA(object):
    def __init__(self, model, decay=0.9999, device=None):
        self.ema = deepcopy(model)
        self.ema.eval()
        self.decay = decay
        self.device = device
        if self.device is not None:
            self.ema.to(device=device)
        self._tab = None
        self._btab = None

    # reference arithmetic: decay * e + (1. - decay) * m, scalars rounded to fp32
    def _scalars(self):
        return float(self.decay), float(1.0 - self.decay)

    def _build_table(self, model, buffers_only=False):
        if buffers_only:
            pairs = [(e, m) for (_, e), (_, m) in zip(self.ema.named_buffers(), model.named_buffers())]
        else:
            pairs = list(zip(self.ema.state_dict().values(), model.state_dict().values()))
        key = (buffers_only,) + tuple((e.data_ptr(), m.data_ptr()) for e, m in pairs)
        cache = self._btab if buffers_only else self._tab
        if cache is not None and cache[0] == key:
            return cache
        esz = _lib.load().es_ema_entry_size()
        raw = bytearray(esz * len(pairs))
        chunks = []
        for j, (e, m) in enumerate(pairs):
            if e.dtype == torch.float32:
                dt = 0
            elif e.dtype == torch.int64:
                dt = 1
            else:
                raise NotImplementedError(f"ModelEMA: unsupported state dtype {e.dtype}")
            if not (e.is_contiguous() and m.is_contiguous()) or m.dtype != e.dtype:
                raise ValueError("ModelEMA expects contiguous state tensors of matching dtype")
            entry = (ctypes.c_void_p(ptr(e)), ctypes.c_void_p(ptr(m)), ctypes.c_long(e.numel()), ctypes.c_int(dt),
                     ctypes.c_int(0))
            buf = b"".join(bytes(x) for x in entry)
            raw[j * esz:j * esz + len(buf)] = buf
            chunks += [(j, c) for c in range((e.numel() + _CHUNK - 1) // _CHUNK)]
        dev = next(iter(self.ema.state_dict().values())).device
        tab = torch.frombuffer(raw, dtype=torch.uint8).to(dev)
        ch = torch.tensor(chunks, dtype=torch.int32).to(dev)
        if buffers_only:
            self._btab = (key, tab, ch)
        else:
            self._tab = (key, tab, ch)
        return (key, tab, ch)

    def _update(self, model, decay, one_minus):
        _, tab, ch = self._build_table(model)
        call("es_ema_update_multi", ptr(tab), ptr(ch), int(ch.shape[0]), decay, one_minus, _lib.stream())
        if hasattr(self.ema, "mark_updated"):
            self.ema.mark_updated()

    def update(self, model):
        d, omd = self._scalars()
        self._update(model, d, omd)

    def update_buffers(self, model):
        """EMA of the buffers only (BatchNorm running stats + num_batches_tracked): the trainers
        fuse the parameters' EMA into the Adam sweep (es_adam_ema_step)."""
        if not any(True for _ in model.named_buffers()):
            return
        d, omd = self._scalars()
        _, tab, ch = self._build_table(model, buffers_only=True)
        call("es_ema_update_multi", ptr(tab), ptr(ch), int(ch.shape[0]), d, omd, _lib.stream())

    def set(self, model):
        # update_fn = lambda e, m: m  ->  0*e + 1*m (exact for finite e)
        with torch.no_grad():
            for e, m in zip(self.ema.state_dict().values(), model.state_dict().values()):
                e.copy_(m)
        if hasattr(self.ema, "mark_updated"):
            self.ema.mark_updated()
