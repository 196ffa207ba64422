#!/bin/bash
# uint8 patch gather through LDS: tests and F1 A/B vs the HEAD library
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; tail -1 "$OUT/$name.log" | cut -c1-120; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
OLD="$GRAFT_REPO_ROOT/build/ab/HEAD/libendossl_hip.so"
ENDOSSL_IM2COL_ROWS=1 run ta 300 $PT -m gpu tests/test_gpu_kernels.py tests/test_gpu_host_input.py -k "im2col or normalisation or host" -x || exit 1
for r in 1 2 3; do
  ENDOSSL_LIB=$OLD run f1o_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  ENDOSSL_IM2COL_ROWS=1 run f1n_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
done
exit 0
