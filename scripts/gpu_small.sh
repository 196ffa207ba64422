#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT -x tests/test_gpu_kernels.py -k "gemm_nt" > gpurun_out/kg.log 2>&1; rc=$?
echo "gemm tests rc=$rc"; tail -2 gpurun_out/kg.log
[ $rc -eq 0 ] || exit 0
for sh in 8 4; do
  timeout -k 10 300 python scripts/gemm_bench.py --shard $sh --variants=-1,0,11,12,5 --rounds 3 --iters 10 --only qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc1_fwd_weak,fc2_dgrad,fc1_dgrad,proj_dgrad,qkv_dgrad > gpurun_out/small_$sh.log 2>&1 || exit 0
  echo "shard $sh"; grep -v amdgpu gpurun_out/small_$sh.log
done
