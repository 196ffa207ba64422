#!/bin/bash
# TN (weight-gradient) kernels: exact-integer tests, microbenchmark of the big-tile variants, F1 bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -6 "$OUT/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run kt 300 $PT -m gpu -x tests/test_gpu_kernels.py -k "gemm_tn"; rc=$?
ok $rc && { run tb 300 python scripts/gemm_bench.py --only fc1_wgrad,fc2_wgrad,qkv_wgrad,proj_wgrad --tn-variants ${TNV:-7,9} --tn-blocks auto --rounds 5; rc=$?; }
for v in ${F1V:-}; do ok $rc && { ENDOSSL_TN_VARIANT=$v run f1_tn$v 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline; rc=$?; }; done
exit 0
