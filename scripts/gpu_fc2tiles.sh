#!/bin/bash
# tile choice for the N = 384 outputs at the train / weak token counts (quantisation over 256 CUs)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python scripts/gemm_bench.py --only fc2_fwd,fc2_fwd_weak,proj_fwd,proj_fwd_weak,proj_dgrad,fc1_dgrad,qkv_dgrad --variants=-1,0,4,10,11,12 --rounds 5 --iters 10 --tn-blocks auto > "$OUT/fc2tiles.log" 2>&1; rc=$?
cat "$OUT/fc2tiles.log" | grep -v "^fc2_wgrad\|^fc1_wgrad\|^qkv_wgrad\|^proj_wgrad"
exit $rc
