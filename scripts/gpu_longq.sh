#!/bin/bash
# long-sequence attention forward (T = 577) with the next query block's Q prefetched: tests, microbench and
# S1, HEAD library vs tree
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1) $(grep -o "\"fwd_occ2\": {[^}]*}" "$OUT/$name.log" | tr "\n" " ")"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
OLD="$GRAFT_REPO_ROOT/build/ab/HEAD/libendossl_hip.so"
run ta 300 $PT -m gpu tests/test_gpu_kernels.py -k "attention or attn" -x || exit 1
for r in 1 2; do
  ENDOSSL_LIB=$OLD run aso_$r 120 python scripts/attn_bench.py --s1 --rounds 3 --iters 5 || exit 1
  run asn_$r 120 python scripts/attn_bench.py --s1 --rounds 3 --iters 5 || exit 1
done
for r in 1 2; do
  ENDOSSL_LIB=$OLD run s1o_$r 300 python bench.py --workload s1 --steps 4 --warmup 2 --no-cpu-baseline || exit 1
  run s1n_$r 300 python bench.py --workload s1 --steps 4 --warmup 2 --no-cpu-baseline || exit 1
done
exit 0
