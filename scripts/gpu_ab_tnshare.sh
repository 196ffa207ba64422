#!/bin/bash
# TN tile / stage variants isolated (asm DMA), then F1 at several weight-gradient CU shares, interleaved twice
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python scripts/gemm_bench.py --only fc1_wgrad,fc2_wgrad,qkv_wgrad --tn-variants 5,6,7,8 --tn-blocks auto --rounds 5 > "$OUT/tnv.log" 2>&1; echo "tnv rc=$?"; grep wgrad "$OUT/tnv.log"
for r in 1 2; do
  for sh in 0.5 0.625 0.75 1.0; do
    ENDOSSL_TN_SHARE=$sh timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/ab_$sh.log" 2>&1 || exit 0
    echo "share $sh: $(grep '^{' "$OUT/ab_$sh.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["mean_launch_ms"], d["roofline"]["isolated"]["mean_launch_ms"])')"
  done
done
exit 0
