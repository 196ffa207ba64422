#!/bin/bash
# round 5: ResNet tests (bf16 maps, graph replay), P0 with bf16 maps vs fp32 maps (ENDOSSL_MAP_BF16=0), both
# graph-replayed, same box interleaved; then a kernel trace of the S1 step
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resnet.py > "$OUT/ty.log" 2>&1; rc=$?; tail -2 "$OUT/ty.log"; [ $rc -ne 0 ] && exit 1
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
for r in 1 2 3; do
  ENDOSSL_MAP_BF16=0 timeout -k 10 200 python -u bench.py --workload p0 --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/y_f32$r.log" 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --workload p0 --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/y_b16$r.log" 2>&1 || exit 1
  echo "p0 r$r fp32maps $(ms $OUT/y_f32$r.log) bf16maps $(ms $OUT/y_b16$r.log)"
done
bash scripts/gpu_r5s1p.sh
