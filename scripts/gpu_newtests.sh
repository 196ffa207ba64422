#!/bin/bash
# The round-3 parity / full-size tests alone, then GEMM calibration (hipBLASLt vs ours at the F1 shapes).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
PT="python -u -m pytest -q -rf -s -p no:cacheprovider --timeout 400 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_blocks.py tests/test_gpu_fullsize.py tests/test_gpu_convs.py > "$OUT/newtests.log" 2>&1; rc=$?
echo "newtests rc=$rc"; grep -E "passed|failed|worst|floor|Error|assert" "$OUT/newtests.log" | tail -12
[ $rc -le 1 ] || exit 0
timeout -k 10 300 python scripts/blas_ref.py > "$OUT/blas.log" 2>&1; echo "blas rc=$?"; cat "$OUT/blas.log" | grep -v amdgpu.ids
