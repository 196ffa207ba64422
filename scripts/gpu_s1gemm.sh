#!/bin/bash
# S1 transformer-branch GEMMs (Conformer-B/384, M = 120 x 577): the DGELU fc2 data gradient against the
# other epilogues on the same shape, per kernel family
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py --s1 --variants=-1,1,6,8,10 --tn-variants 7 --tn-blocks auto \
  --only fc2_dgrad_dgelu,fc1_fwd_gelu,fc2_dgrad_plain,fc2_dgrad,fc1_fwd --rounds 3 > gpurun_out/s1gemm.log 2>&1
rc=$?; tail -6 gpurun_out/s1gemm.log; exit $rc
