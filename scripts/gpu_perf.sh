#!/bin/bash
# Kernel A/B pass: attention tests (incl. the persistent forward), attention / TN microbenchmarks,
# F1 bench with each attention forward variant.  Each GPU step has its own time limit.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -4 "$OUT/$name.log"
  return $rc
}
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run ka 300 $PT -m gpu -x tests/test_gpu_kernels.py -k "attention"; rc=$?
ok $rc && { run ab 200 python scripts/attn_bench.py; rc=$?; }
ok $rc && { run tb 300 python scripts/gemm_bench.py --only ${TN_ONLY:-fc1_wgrad,fc2_wgrad,qkv_wgrad,proj_wgrad} --tn-variants ${TN_VARIANTS:-5,6,7,8} --tn-blocks ${TN_BLOCKS:-auto} --rounds 5; rc=$?; }
for v in ${F1_ATTN:-2 4}; do
  ok $rc && { ENDOSSL_ATTN_VARIANT=$v run f1_attn$v 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline; rc=$?; }
done
exit 0
