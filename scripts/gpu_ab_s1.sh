#!/bin/bash
# S1 A/B over ABV env settings (interleaved twice)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
i=0
for r in 1 2; do for e in $ABV; do
  i=$((i+1))
  env $(echo $e | tr "," " ") timeout -k 10 400 python bench.py --workload s1 --steps 3 --warmup 2 > "$OUT/abs1_$i.log" 2>&1 || exit 1
  echo "$e $(tail -1 $OUT/abs1_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done
exit 0
