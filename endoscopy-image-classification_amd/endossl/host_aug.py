"""Host-side input path: the reference's training transforms on the host,
native, feeding the device's uint8 patch gather.

The reference builds its SSL batches with torchvision / PIL transforms in DataLoader workers
(`code/dataset.py:24-56` TransformFixMatch, `:185-207` the labeled train transform,
`code/randaugment.py:207-222` RandAugmentMC) and normalises to fp32 on the host.  Here the same
transforms run in C++ (`csrc/host_aug.cpp`, C-ABI `include/endossl_host.h`, `libendossl_host.so`)
on a pool of host threads and write planar uint8 batches into pinned memory; ToTensor + Normalize
happen on the device inside the patch gather (`es_patch_im2col_u8`), so the host never makes fp32
and the H2D copy is a quarter of the fp32 bytes.

  TransformFixMatchNative(config)(pil_image) -> (weak, strong) uint8 [3, S, S] tensors
  HostBatcher(images, ...) -> pinned uint8 [n, 3, S, S] batches, copied to the device on a side stream

Parity: every PIL op is pinned bit-exact to PIL itself (tests/test_host_aug.py); the random
parameters follow the reference's distributions on the library's own per-image streams (the
reference's Python / numpy / torch generator streams are not reproduced).
"""
import ctypes
import os
import threading

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ENDOSSL_HOST_LIB", os.path.join(_HERE, "lib", "libendossl_host.so"))
ABI_VERSION = 2

# fixmatch_augment_pool() order (code/randaugment.py:147-163)
POOL = ("AutoContrast", "Brightness", "Color", "Contrast", "Equalize", "Identity", "Posterize", "Rotate",
        "Sharpness", "ShearX", "ShearY", "Solarize", "TranslateX", "TranslateY")
ENHANCE = {"brightness": 0, "color": 1, "contrast": 2, "sharpness": 3}

_P = ctypes.c_void_p
_I = ctypes.c_int
_SIG = {
    "esh_abi_version": (_I, []),
    "esh_aug_op": (_I, [_I, _P, _P, _I, _I, _I, _I]),
    "esh_enhance": (_I, [_I, _P, _P, _I, _I, ctypes.c_float]),
    "esh_color_op": (_I, [_I, _P, _P, _I, _I, ctypes.c_double]),
    "esh_rotate": (_I, [_P, _P, _I, _I, ctypes.c_double]),
    "esh_resize_bilinear": (_I, [_P, _I, _I, _P, _I, _I]),
    "esh_fill_rect": (_I, [_P, _I, _I, _I, _I, _I, _I, _I]),
    "esh_pad_reflect_crop": (_I, [_P, _I, _I, _I, _I, _I, _I, _P]),
    "esh_transform_batch": (_I, [_I, ctypes.POINTER(_P), ctypes.POINTER(_I), ctypes.POINTER(_I), _I, _I, _I,
                                 ctypes.c_uint64, _I, _P, _P, _P]),
}
_lib = None
_lock = threading.Lock()


class HostLibraryError(RuntimeError):
    pass


def load():
    """libendossl_host.so with its signatures bound (built by `make` in csrc/, or __graft_entry__.build())."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HostLibraryError(f"{LIB_PATH} missing: run `make` in csrc/ (or __graft_entry__.build())")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIG.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            if lib.esh_abi_version() != ABI_VERSION:
                raise HostLibraryError(f"host ABI {lib.esh_abi_version()} != {ABI_VERSION}")
            _lib = lib
    return _lib


def _check(rc, name):
    if rc != 0:
        raise HostLibraryError(f"{name} failed with status {rc}")


def _hwc(img):
    """RGB image (PIL or HWC uint8 array) -> C-contiguous HWC uint8 numpy array."""
    a = np.asarray(img.convert("RGB") if hasattr(img, "convert") else img)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"expected an RGB HWC uint8 image, got {a.dtype} {a.shape}")
    return np.ascontiguousarray(a)


def _ptr(a):
    return a.ctypes.data_as(_P)


# ---- single ops (the reference's augment pool, for tests and custom pipelines) -----------------
def aug_op(img, op, v, neg=False):
    """Pool op `op` (name or index) at magnitude v on one image; neg = the op's sign draw."""
    a = _hwc(img)
    k = POOL.index(op) if isinstance(op, str) else int(op)
    out = np.empty_like(a)
    _check(load().esh_aug_op(k, _ptr(a), _ptr(out), a.shape[1], a.shape[0], int(v), int(bool(neg))), "esh_aug_op")
    return out


def enhance(img, kind, factor):
    a = _hwc(img)
    out = np.empty_like(a)
    _check(load().esh_enhance(ENHANCE[kind], _ptr(a), _ptr(out), a.shape[1], a.shape[0], float(factor)), "esh_enhance")
    return out


def adjust_hue(img, factor):
    a = _hwc(img)
    out = np.empty_like(a)
    _check(load().esh_color_op(0, _ptr(a), _ptr(out), a.shape[1], a.shape[0], float(factor)), "esh_color_op")
    return out


def grayscale3(img):
    a = _hwc(img)
    out = np.empty_like(a)
    _check(load().esh_color_op(1, _ptr(a), _ptr(out), a.shape[1], a.shape[0], 0.0), "esh_color_op")
    return out


def rotate(img, angle):
    a = _hwc(img)
    out = np.empty_like(a)
    _check(load().esh_rotate(_ptr(a), _ptr(out), a.shape[1], a.shape[0], float(angle)), "esh_rotate")
    return out


def resize_bilinear(img, size):
    """Image.resize(size=(w, h), BILINEAR)."""
    a = _hwc(img)
    w, h = size
    out = np.empty((h, w, 3), np.uint8)
    _check(load().esh_resize_bilinear(_ptr(a), a.shape[1], a.shape[0], _ptr(out), w, h), "esh_resize_bilinear")
    return out


def fill_rect(img, xy, v=127):
    a = _hwc(img).copy()
    _check(load().esh_fill_rect(_ptr(a), a.shape[1], a.shape[0], *[int(t) for t in xy], int(v)), "esh_fill_rect")
    return a


def pad_reflect_crop(img, pad, top, left, size):
    a = _hwc(img)
    out = np.empty((size, size, 3), np.uint8)
    _check(load().esh_pad_reflect_crop(_ptr(a), a.shape[1], a.shape[0], pad, top, left, size, _ptr(out)),
           "esh_pad_reflect_crop")
    return out


# ---- batches --------------------------------------------------------------------------------------
KINDS = {"fixmatch": (0, 2), "labeled": (1, 1), "comatch": (2, 3), "eval": (3, 1)}  # kind -> (id, outputs)


def transform_batch(images, size, kind="fixmatch", is_crop=True, seed=0, threads=None, outs=None):
    """Run one of the reference's transforms over a list of RGB images on `threads` host threads.

    kind 'fixmatch': TransformFixMatch (code/dataset.py:24-56) -> (weak, strong); 'comatch':
    TransformCoMatch (:58-110) -> (weak, strong_0, strong_1); 'labeled': the labeled train transform
    (:185-207) -> (x,); 'eval': Resize -> CenterCrop (:217-231) -> (x,).  Each output uint8
    [n, 3, S, S]; `outs` may hold preallocated (e.g. pinned) CPU tensors.  Image i's randomness is
    keyed on (seed, i) only."""
    arrs = [_hwc(im) for im in images]
    n = len(arrs)
    k, nout = KINDS[kind]
    shape = (n, 3, size, size)
    outs = list(outs) if outs is not None else [torch.empty(shape, dtype=torch.uint8) for _ in range(nout)]
    if len(outs) != nout:
        raise ValueError(f"kind {kind!r} writes {nout} outputs")
    for t in outs:
        if tuple(t.shape) != shape or t.dtype != torch.uint8 or not t.is_contiguous() or t.device.type != "cpu":
            raise ValueError(f"output must be a contiguous CPU uint8 tensor of shape {shape}")
    ptrs = (_P * n)(*[a.ctypes.data for a in arrs])
    ws = (_I * n)(*[a.shape[1] for a in arrs])
    hs = (_I * n)(*[a.shape[0] for a in arrs])
    threads = threads or min(16, os.cpu_count() or 1)
    op = [t.data_ptr() for t in outs] + [None] * (3 - nout)
    rc = load().esh_transform_batch(k, ptrs, ws, hs, n, size, int(bool(is_crop)), int(seed) & (2 ** 64 - 1),
                                    int(threads), *op)
    _check(rc, "esh_transform_batch")
    return tuple(outs)


class TransformFixMatchNative:
    """Drop-in for the reference's TransformFixMatch(config, mean, std) (code/dataset.py:24-56), minus
    the normalisation (done on the device): __call__(img) -> (weak, strong) uint8 [3, S, S]."""

    def __init__(self, config, mean=None, std=None, seed=0):
        self.size = int(config.DATA.IMG_SIZE)
        self.is_crop = bool(getattr(config.DATA, "IS_CROP", True))
        self.seed = seed
        self.calls = 0

    def __call__(self, x):
        w, s = transform_batch([x], self.size, "fixmatch", self.is_crop, seed=self.seed + self.calls, threads=1)
        self.calls += 1
        return w[0], s[0]


class HostBatcher:
    """Double-buffered host producer: builds batch k+1 (uint8, pinned) on host threads while batch k is
    consumed, and copies it to the device on a side stream (code/dataset.py's DataLoader role).

    images: list of RGB images (PIL or HWC uint8); each batch draws `batch` of them uniformly (with a
    fresh per-batch seed) and next() returns the kind's views as device uint8 [batch, 3, S, S] tensors
    ('fixmatch': (weak, strong), 'comatch': (weak, strong_0, strong_1), 'labeled' / 'eval': (x,)),
    ready for es_patch_im2col_u8."""

    def __init__(self, images, batch, size, kind="fixmatch", is_crop=True, seed=0, threads=None, device="cuda"):
        self.images = [_hwc(im) for im in images]
        self.batch, self.size, self.kind, self.is_crop = batch, size, kind, is_crop
        self.seed, self.threads, self.device = seed, threads, device
        self.step = 0
        nout = KINDS[kind][1]
        pin = torch.cuda.is_available() and str(device).startswith("cuda")
        shape = (batch, 3, size, size)
        self._host = [[torch.empty(shape, dtype=torch.uint8, pin_memory=pin) for _ in range(nout)] for _ in range(2)]
        self._stream = torch.cuda.Stream(device=device) if pin else None
        self._events = [None, None]
        self._worker = None
        self._error = None
        self._submit(0)

    def _indices(self, step):
        g = np.random.default_rng((self.seed, step))
        return g.integers(0, len(self.images), self.batch)

    def _build(self, step):
        try:
            slot = step & 1
            if self._events[slot] is not None:  # the copy out of this slot two batches ago must be done
                self._events[slot].synchronize()
            idx = self._indices(step)
            transform_batch([self.images[i] for i in idx], self.size, self.kind, self.is_crop,
                            seed=(self.seed << 32) ^ step, threads=self.threads, outs=self._host[slot])
        except BaseException as e:  # surfaced by next()
            self._error = e

    def _submit(self, step):
        self._worker = threading.Thread(target=self._build, args=(step,), daemon=True)  # ctypes drops the GIL
        self._worker.start()

    def next(self):
        """The next batch on the device (the copy is ordered before any later work on the caller's stream)."""
        self._worker.join()
        if self._error is not None:
            raise self._error
        slot = self.step & 1
        bufs = self._host[slot]
        if self._stream is None:
            out = tuple(b.clone() for b in bufs)
        else:
            cur = torch.cuda.current_stream(self.device)
            self._stream.wait_stream(cur)
            with torch.cuda.stream(self._stream):
                out = tuple(b.to(self.device, non_blocking=True) for b in bufs)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            self._events[slot] = ev
            cur.wait_stream(self._stream)
            for d in out:
                d.record_stream(cur)
        self.step += 1
        self._submit(self.step)
        return out
