#!/bin/bash
# round 5: the supervised step's hipGraph replay (SupLearning.use_graph): ResNet / trainer tests, then P0
# graph vs eager (same tree, interleaved)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resnet.py > "$OUT/ty.log" 2>&1; rc=$?; tail -2 "$OUT/ty.log"; [ $rc -ne 0 ] && exit 1
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
for r in 1 2 3; do
  line="p0 r$r"
  for gr in off on; do
    timeout -k 10 200 python -u bench.py --workload p0 --steps 100 --warmup 10 --no-cpu-baseline --graph $gr > "$OUT/y_$gr$r.log" 2>&1 || exit 1
    line="$line $gr $(ms $OUT/y_$gr$r.log)"
  done
  echo "$line"
done
