#!/bin/bash
# S1 transformer-branch NT GEMMs: per-shape variant sweep (isolated)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_bench.py --s1 --variants=${V:--1,6,10,0,1,2,5,16,18} --rounds 3 --tn-variants 0 --only ${ONLY:-fc2_dgrad,fc1_fwd,qkv_fwd,fc2_fwd,fc1_dgrad,qkv_dgrad,proj_fwd,proj_dgrad} > "$OUT/s1nt.log" 2>&1; rc=$?
grep -v "^#\|amdgpu.ids" "$OUT/s1nt.log" | cut -c1-600; exit $rc
