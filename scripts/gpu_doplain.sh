#!/bin/bash
# plain C stores for the proj data gradient's output (dO, 77 MB, read by the attention backward next)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; return $rc; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
for r in 1 2 3; do
  run o_$r 200 $B || exit 1
  ENDOSSL_DO_PLAIN=1 run n_$r 200 $B || exit 1
done
exit 0
