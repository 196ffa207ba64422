#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py --s1 --only fc2_dgrad_dgelu,fc2_dgrad,fc1_fwd_gelu,fc2_dgrad_plain,fc1_fwd --variants=-1,0,1,2,6,10 --rounds 3 --iters 5 > gpurun_out/dgelu.log 2>&1; echo rc=$?
cat gpurun_out/dgelu.log | grep -v amdgpu
