#!/bin/bash
# re-sweep of the block weight-gradient CU share (ENDOSSL_LAYER_TN_SHARE) after the attention changes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; return $rc; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
for r in 1 2; do
  for sh in 0.3125 0.375 0.4375 0.5; do ENDOSSL_LAYER_TN_SHARE=$sh run s${sh}_$r 200 $B || exit 1; done
done
exit 0
