#!/bin/bash
# NT GEMM variants: exact-integer / epilogue tests, microbenchmark at the F1 (and S1) shapes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-12} "$OUT/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run kn 300 $PT -m gpu -x tests/test_gpu_kernels.py -k "gemm_nt"; rc=$?
ok $rc && { run nb 300 python scripts/gemm_bench.py --variants=${NTV:--1,10} --tn-variants 7 --only ${ONLY:-qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc1_fwd_weak,fc2_dgrad,fc1_dgrad,proj_dgrad,qkv_dgrad} --rounds 5; rc=$?; }
ok $rc && [ -n "$S1" ] && { run nbs 300 python scripts/gemm_bench.py --s1 --variants=${NTV:--1,10} --tn-variants 7 --only qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc2_dgrad,fc1_dgrad,proj_dgrad,qkv_dgrad --rounds 3; rc=$?; }
exit 0
