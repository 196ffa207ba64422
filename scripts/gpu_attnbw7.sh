#!/bin/bash
# attention backward with seven waves per workgroup (variant 4) vs the 4-wave pair kernels (3): microbench
# + bit-exactness, F1 A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1) $(grep -o "\"bwd_dq2_dkv2\": {[^}]*}\|\"bwd_w7\": {[^}]*}\|w7 == plain: [A-Za-z]*" "$OUT/$name.log" | tr "\n" " ")"; return $rc; }
run ab1 120 python scripts/attn_bench.py --rounds 5 --iters 10 || exit 1
run ab2 120 python scripts/attn_bench.py --rounds 5 --iters 10 || exit 1
for r in 1 2; do
  run f1o_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  ENDOSSL_ATTN_BWD_VARIANT=4 run f1n_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
done
exit 0
