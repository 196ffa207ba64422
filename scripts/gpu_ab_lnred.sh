#!/bin/bash
# LayerNorm backward: dgamma / dbeta reductions in one launch; tests, N = 8 shard and F1, HEAD library vs tree
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
OLD="$GRAFT_REPO_ROOT/build/ab/HEAD/libendossl_hip.so"
run tk 400 $PT -m gpu tests/test_gpu_kernels.py tests/test_gpu_step.py tests/test_gpu_blocks.py -x || exit 1
for r in 1 2 3; do
  ENDOSSL_LIB=$OLD run b8o_$r 200 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  run b8n_$r 200 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
for r in 1 2; do
  ENDOSSL_LIB=$OLD run f1o_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  run f1n_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
done
exit 0
