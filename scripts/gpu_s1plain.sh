#!/bin/bash
# S1: plain C stores for the D = 768 residual outputs (256x256 tile) vs nt
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; return $rc; }
B="python bench.py --workload s1 --steps 4 --warmup 2 --no-cpu-baseline"
for r in 1 2; do
  run o_$r 300 $B || exit 1
  ENDOSSL_S1_PLAIN=1 run n_$r 300 $B || exit 1
done
exit 0
