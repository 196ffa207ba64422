#!/bin/bash
# same-box P0 A/B: abtree/ (older commit) vs this tree, and this tree with one conv / BatchNorm knob flipped
# (KNOB=value through the C ABI before bench.py runs); interleaved R rounds, more steps than the default P0 line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
KN="import os, sys, runpy; sys.argv = ['bench.py'] + sys.argv[1:]; sys.path.insert(0, 'endoscopy-image-classification_amd')
from endossl import _lib; L = _lib.load(); k, v = os.environ['KNOB'].split('='); print(k, getattr(L, k)(int(v)))
runpy.run_path('bench.py', run_name='__main__')"
A="--workload p0 --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline ${BARGS}"
for r in $(seq ${R:-3}); do
  timeout -k 10 200 python -u abtree/bench.py $A > "$OUT/x_old$r.log" 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py $A > "$OUT/x_new$r.log" 2>&1 || exit 1
  line="p0 r$r old $(ms $OUT/x_old$r.log) new $(ms $OUT/x_new$r.log)"
  i=0
  for kv in ${KNOBS:-es_set_conv_ring=0 es_set_bn_cs=0}; do
    i=$((i+1)); KNOB=$kv timeout -k 10 200 python -u -c "$KN" $A > "$OUT/x_k$i$r.log" 2>&1 || exit 1
    line="$line $kv $(ms $OUT/x_k$i$r.log)"
  done
  echo "$line"
done
