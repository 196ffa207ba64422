#!/bin/bash
# N=8 shard (B=8, mu=7 per rank on one GPU): whole-axis grouped weight gradients (default) vs the per-block
# split-K grouped launch at several CU shares
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"; return $rc; }
B="python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline"
for r in 1 2; do
  run d_$r 200 $B || exit 1
  for sh in 0.375 0.5 0.75 1.0; do
    ENDOSSL_GROUP_WGRAD=0 ENDOSSL_TN_SHARE_MIN_M=8192 ENDOSSL_LAYER_TN_SHARE=$sh run l${sh}_$r 200 $B || exit 1
  done
done
exit 0
