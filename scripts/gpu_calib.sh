#!/bin/bash
# Calibration: hipBLASLt (torch bf16 matmul) vs this library's default kernels at the F1 GEMM shapes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python scripts/blas_ref.py > "$OUT/blas.log" 2>&1; echo "blas rc=$?"; grep -v amdgpu.ids "$OUT/blas.log"
timeout -k 10 300 python scripts/gemm_bench.py --variants ${VARIANTS:--1} --tn-variants ${TN_VARIANTS:--1} --tn-blocks ${TN_BLOCKS:-auto} --rounds 3 > "$OUT/gb.log" 2>&1; echo "gemm bench rc=$?"; cat "$OUT/gb.log"
