#!/bin/bash
# round 4: the activation-stationary K = 384 GEMM (variant 30) -- bit-identity tests, then the isolated
# F1-shape microbenchmark against the per-shape defaults (NOTEST=1: the benchmark alone)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > "$OUT/panel_t.log" 2>&1; rc=$?
  echo "tests rc=$rc"; tail -5 "$OUT/panel_t.log"
  [ $rc -ne 0 ] && exit 1
fi
timeout -k 10 300 python -u scripts/gemm_bench.py --variants=${VARIANTS:--1,30} --rounds 5 --only ${ONLY:-qkv_fwd,proj_fwd,fc1_fwd,fc1_fwd_weak,fc2_dgrad,proj_dgrad,qkv_fwd_weak,proj_fwd_weak} > "$OUT/panel_b.log" 2>&1; rc=$?
echo "bench rc=$rc"; cat "$OUT/panel_b.log"
exit $rc
