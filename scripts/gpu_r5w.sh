#!/bin/bash
# same-box A/B: the tree at an older commit (abtree/, made by `git archive <ref> bench.py <pkg>` + make) vs this tree,
# interleaved R rounds over F1 / P0 / the N = 8 shard; DEFER=0 arm: this tree with the deferred LayerNorm grads off
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
ND="import sys, runpy; sys.argv = ['bench.py'] + sys.argv[1:]; sys.path.insert(0, 'endoscopy-image-classification_amd')
import endossl.vit as v; v.Engine.DEFER_LN_GRADS = False
runpy.run_path('bench.py', run_name='__main__')"
for r in 1 2 3; do
  for w in f1 p0 sh; do
    case $w in f1) a="--steps 100 --warmup 5";; p0) a="--workload p0 --steps 20 --warmup 5";; sh) a="--batch 8 --steps 50 --warmup 10";; esac
    timeout -k 10 200 python -u abtree/bench.py --no-cpu-baseline $a > "$OUT/w_old_$w$r.log" 2>&1 || exit 1
    timeout -k 10 200 python -u bench.py --no-cpu-baseline $a > "$OUT/w_new_$w$r.log" 2>&1 || exit 1
    line="$w r$r old $(ms $OUT/w_old_$w$r.log) new $(ms $OUT/w_new_$w$r.log)"
    if [ $w != p0 ]; then timeout -k 10 200 python -u -c "$ND" --no-cpu-baseline $a > "$OUT/w_nd_$w$r.log" 2>&1 || exit 1; line="$line nodefer $(ms $OUT/w_nd_$w$r.log)"; fi
    echo "$line"
  done
done
