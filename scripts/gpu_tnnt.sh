#!/bin/bash
# grouped weight-gradient launch: operand DMA with the nt cache policy (ENDOSSL_TN_VARIANT=20) vs default
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep '^{' "$OUT/$name.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_step"], r["mean_launch_ms"], r["isolated"]["mean_launch_ms"])')"; return $rc; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
for r in 1 2 3; do
  run d_$r 200 $B || exit 1
  ENDOSSL_TN_VARIANT=20 run nt_$r 200 $B || exit 1
done
exit 0
