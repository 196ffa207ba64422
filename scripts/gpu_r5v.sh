#!/bin/bash
# round 5: the bf16 convs' 64-channel tile on small grids (es_set_conv_small): ResNet tests, then P0 with the
# knob at 128 (default) / 256 / 512, same box, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resnet.py tests/test_gpu_convs.py > "$OUT/tv.log" 2>&1; rc=$?; tail -2 "$OUT/tv.log"; [ $rc -ne 0 ] && exit 1
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
KN="import os, sys, runpy; sys.argv = ['bench.py'] + sys.argv[1:]; sys.path.insert(0, 'endoscopy-image-classification_amd')
from endossl import _lib; L = _lib.load(); k, v = os.environ['KNOB'].split('='); getattr(L, k)(int(v))
runpy.run_path('bench.py', run_name='__main__')"
for r in 1 2 3; do
  line="p0 r$r"
  for v in 128 256 512; do
    KNOB=es_set_conv_small=$v timeout -k 10 200 python -u -c "$KN" --workload p0 --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/v_p0_$v$r.log" 2>&1 || exit 1
    line="$line $v $(ms $OUT/v_p0_$v$r.log)"
  done
  echo "$line"
done
