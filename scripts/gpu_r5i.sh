#!/bin/bash
# round 5: the small shard's two-lane data-gradient chain (Engine.SHARD_LANES): step tests (lanes vs one lane,
# grouped vs split-K, pruned vs full rows, graph replay), the per-op shard parity, then the shard A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
run tstep 600 $PT tests/test_gpu_step.py tests/test_gpu_blocks.py tests/test_gpu_dist.py || exit 1
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
off="import sys; sys.argv=['bench.py','--batch','8','--steps','200','--warmup','10','--no-cpu-baseline']; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.vit as v; v.Engine.SHARD_LANES=False; import runpy; runpy.run_path('bench.py', run_name='__main__')"
for r in 1 2 3; do
  timeout -k 10 200 python -u -c "$off" > "$OUT/la$r.log" 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --batch 8 --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/lb$r.log" 2>&1 || exit 1
  echo "shard round $r: one lane $(ms $OUT/la$r.log)  two lanes $(ms $OUT/lb$r.log)"
done
