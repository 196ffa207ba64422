#!/bin/bash
# NT kernel sweep (every family, nt C stores) at the F1 shapes and at a rank's shard (N = 2, 4, 8)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_nt" > "$OUT/nts_t.log" 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 "$OUT/nts_t.log"
[ $rc -eq 0 ] || exit 0
for SH in 1 2 4 8; do
timeout -k 10 300 python scripts/gemm_bench.py --variants=${VARIANTS:--1,0,2,5,6,10,11,12} --tn-variants 7 --tn-blocks auto --rounds 3 --shard $SH --only ${ONLY:-qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc1_fwd_weak,fc2_dgrad,fc1_dgrad,proj_dgrad,qkv_dgrad,qkv_fwd_weak,proj_fwd_weak,fc2_fwd_weak} > "$OUT/nts_b$SH.log" 2>&1; echo "bench shard $SH rc=$?"; grep -v amdgpu.ids "$OUT/nts_b$SH.log"
done
