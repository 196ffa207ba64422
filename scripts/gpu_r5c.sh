#!/bin/bash
# round 5: NT kernel-family sweep at every F1 shape (isolated, interleaved rounds in one process)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 500 python3 scripts/gemm_bench.py --variants=-1,0,1,2,5,6,10,11 --rounds 5 --iters 10 \
  --only qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc1_fwd_weak,fc2_dgrad,fc1_dgrad,proj_dgrad,qkv_dgrad,qkv_fwd_weak,proj_fwd_weak,fc2_fwd_weak \
  > "$OUT/sweep.log" 2>&1; rc=$?; tail -14 "$OUT/sweep.log"; exit $rc
