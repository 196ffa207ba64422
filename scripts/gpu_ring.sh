#!/bin/bash
# ring NT kernel: GEMM tests for the persistent variants, then the F1 NT shapes vs the defaults
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_nt and (v21 or v22 or v23 or v24 or auto or v10 or v25 or v26 or v27 or v28)" > "$OUT/ring_t.log" 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 "$OUT/ring_t.log"
[ $rc -eq 0 ] || exit 0
timeout -k 10 300 python scripts/gemm_bench.py --variants=${VARIANTS:--1,25,26,27} --tn-variants 7 --tn-blocks auto --rounds 3 --only ${ONLY:-qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc1_fwd_weak,fc2_dgrad,fc1_dgrad,proj_dgrad,qkv_dgrad} > "$OUT/ring_b.log" 2>&1; echo "bench rc=$?"; grep -v amdgpu.ids "$OUT/ring_b.log"
