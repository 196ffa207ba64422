#!/bin/bash
# GEMM kernel tests (both variants) + GEMM microbenchmark
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -rf -p no:cacheprovider -k "gemm or layernorm or attention" > "$OUT/kg.log" 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -3 "$OUT/kg.log"
[ $rc -le 1 ] && { timeout -k 10 400 python scripts/gemm_bench.py --variants ${VARIANTS:-1,2,5} --tn-variants ${TN_VARIANTS:-0,1,2,3,4} --rounds 3 > "$OUT/gb.log" 2>&1; echo "gemm bench rc=$?"; cat "$OUT/gb.log"; }
exit 0
