#!/bin/bash
# per-layer grouped weight gradients: kernel tests, F1 A/B (per-GEMM vs per-layer launches, interleaved),
# CU-share sweep, then the PMC passes of the grouped launch
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run kt 300 $PT -m gpu tests/test_gpu_kernels.py -k "tn" || exit 1
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
for r in 1 2; do
  ENDOSSL_LAYER_WGRAD=0 run ab0_$r 200 $B || exit 1
  ENDOSSL_LAYER_WGRAD=1 run ab1_$r 200 $B || exit 1
done
for sh in 0.375 0.625 0.75; do ENDOSSL_LAYER_TN_SHARE=$sh run sh_$sh 200 $B || exit 1; done
run shard4 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --batch 16 || exit 1
ENDOSSL_LAYER_WGRAD=0 run shard4_0 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --batch 16 || exit 1
run ts 400 $PT -m gpu tests/test_gpu_step.py tests/test_gpu_blocks.py -x || exit 1
bash scripts/gpu_pmc_step.sh
exit 0
