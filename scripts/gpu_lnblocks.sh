#!/bin/bash
# LayerNorm backward workgroup count (ENDOSSL_LN_BWD_BLOCKS) in the F1 step and the N = 8 shard
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; return $rc; }
for r in 1 2; do
  for b in 512 1024 2048; do ENDOSSL_LN_BWD_BLOCKS=$b run f${b}_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1; done
done
for b in 512 1024 2048; do ENDOSSL_LN_BWD_BLOCKS=$b run s$b 200 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1; done
exit 0
