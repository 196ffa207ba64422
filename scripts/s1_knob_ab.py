"""One S1 bench line with a C-ABI tuning knob set first (A/B runs of library knobs without an environment
variable): python scripts/s1_knob_ab.py es_set_conv_dw_target 1024 [bench args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
from endossl import _lib  # noqa: E402

knob, val = sys.argv[1], int(sys.argv[2])
old = getattr(_lib.load(), knob)(val)
print(f"{knob}({val}) (was {old})", file=sys.stderr, flush=True)
sys.argv = ["bench.py"] + (sys.argv[3:] or ["--workload", "s1", "--steps", "3", "--warmup", "2", "--no-cpu-baseline"])
import bench  # noqa: E402

bench.main()
