#!/bin/bash
# round 5: the S1 (Conformer-B/384 transformer branch) NT shapes per kernel family, isolated
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 500 python3 scripts/gemm_bench.py --s1 --variants=-1,0,1,2,6,10 --rounds 3 --iters 5 \
  --only qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc2_dgrad,fc1_dgrad,qkv_dgrad,fc2_dgrad_plain > "$OUT/s1sweep.log" 2>&1; rc=$?; tail -9 "$OUT/s1sweep.log"; exit $rc
