#!/bin/bash
# round 4: GEMM kernel tests (incl. the panel kernel's bit-identity), the S1 per-op parity, the panel bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 "$OUT/$name.log" | cut -c1-400; return $rc; }
run kg 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" || exit 1
run pb 300 python -u scripts/gemm_bench.py --variants=-1,30 --rounds 5 --only qkv_fwd,fc1_fwd,fc1_fwd_weak,fc2_dgrad,proj_dgrad,qkv_fwd_weak || exit 1
cat "$OUT/pb.log"
run s1 400 python -u -m pytest tests/test_gpu_s1_blocks.py -x -q -rf -s -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
exit 0
