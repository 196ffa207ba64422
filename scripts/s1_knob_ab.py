"""One bench line with C-ABI tuning knobs (or package module constants) set first (A/B runs of library knobs without environment variables):
  python scripts/s1_knob_ab.py es_set_conv_dw_target=1024 [es_set_...=v ...] [bench args...]
(no bench args: the S1 workload, 3 steps after 2 warm-up)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
from endossl import _lib  # noqa: E402

args = sys.argv[1:]
while args and "=" in args[0] and (args[0].startswith("es_") or args[0].startswith("endossl.")):
    knob, val = args.pop(0).split("=")
    if knob.startswith("es_"):
        old = getattr(_lib.load(), knob)(int(val))
    else:  # a module constant of the package, e.g. endossl.conformer.BN_Y_FREE=0
        import importlib
        mod, attr = knob.rsplit(".", 1)
        try:
            m = importlib.import_module(mod)
        except ModuleNotFoundError:  # a class attribute, e.g. endossl.vit.Engine.TN_SHARE=0.5
            pm, cls = mod.rsplit(".", 1)
            m = getattr(importlib.import_module(pm), cls)
        old = getattr(m, attr)
        setattr(m, attr, type(old)(float(val)) if isinstance(old, float) else type(old)(int(val)))
    print(f"{knob}={val} (was {old})", file=sys.stderr, flush=True)
sys.argv = ["bench.py"] + (args or ["--workload", "s1", "--steps", "3", "--warmup", "2", "--no-cpu-baseline"])
import bench  # noqa: E402

bench.main()
