#!/bin/bash
# in-step A/B: F1 (B=64) and the per-rank shards (B=32/16/8) under each env setting of ABV, interleaved twice
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
i=0
for r in 1 2; do for B in ${BATCHES:-64 32 16 8}; do for e in $ABV; do
  i=$((i+1))
  env $(echo $e | tr "," " ") timeout -k 10 300 python bench.py --batch $B --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline > "$OUT/abst$i.log" 2>&1 || { echo "run $i failed"; tail -3 "$OUT/abst$i.log"; exit 1; }
  echo "B=$B $e $(tail -1 $OUT/abst$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done; done
exit 0
