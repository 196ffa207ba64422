"""endossl -- MI355X-native FixMatch SSL training step (drop-in for taindp98/Endoscopy-Image-Classification's
code/fixmatch.py + code/build.py surfaces).  Compute runs in libendossl_hip.so (gfx950) through the
C-ABI of include/endossl.h; there is no CPU fallback.
"""
from .utils import AttrDict, AverageMeter, get_config, count_parameters  # noqa: F401

__all__ = ["AttrDict", "AverageMeter", "get_config", "count_parameters"]
