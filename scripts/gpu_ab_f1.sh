#!/bin/bash
# F1 A/B over an environment knob: ABV="VAR=a VAR=b" runs bench.py under each, interleaved twice
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
i=0
for r in 1 2; do for e in $ABV; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/ab$i.log" 2>&1 || exit 1
  echo "$e $(tail -1 $OUT/ab$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done
exit 0
