#!/bin/bash
# TN weight-gradient probes at the F1 fc1 / fc2 sites: big-tile variants 7 (64x2), 8 (32x4) and the
# stream-alone / MFMA-alone probes (10/11 = 64x2, 12/13 = 32x4), whole chip (s32) and half chip (s16)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py --variants=-1 --only fc1_wgrad,fc2_wgrad,qkv_wgrad \
  --tn-variants 7,8,10,11,12,13 --tn-blocks s32,s16 --rounds 3 > gpurun_out/tnprobe.log 2>&1
rc=$?; tail -5 gpurun_out/tnprobe.log; exit $rc
