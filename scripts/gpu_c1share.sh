#!/bin/bash
# C1: CU share of the grouped block weight gradients (C1's main stream is its critical path)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"; return $rc; }
for r in 1 2; do
  for sh in 0.1875 0.25 0.3125 0.375; do
    ENDOSSL_LAYER_TN_SHARE=$sh run c1_${sh}_$r 300 python bench.py --workload c1 --steps 5 --warmup 2 || exit 1
  done
done
exit 0
