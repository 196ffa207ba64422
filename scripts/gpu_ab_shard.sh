#!/bin/bash
# per-rank shard A/B: bench.py --batch $BATCH (the global B of one rank's share) under each env setting of ABV
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
i=0
for r in 1 2; do for e in $ABV; do
  i=$((i+1))
  env $(echo $e | tr "," " ") timeout -k 10 300 python bench.py --batch ${BATCH:-32} --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/abs$i.log" 2>&1 || exit 1
  echo "B=${BATCH:-32} $e $(tail -1 $OUT/abs$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done
exit 0
