#!/bin/bash
# dK/dV pass with the next key pair's rows prefetched: tests, microbench (F1 / S1 shapes), F1 A/B vs HEAD library
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1) $(grep -o "\"bwd_dq2_dkv2\": {[^}]*}\|dq2 + dkv2 == plain: [A-Za-z]*" "$OUT/$name.log" | tr "\n" " ")"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
OLD="$GRAFT_REPO_ROOT/build/ab/HEAD/libendossl_hip.so"
run ta 300 $PT -m gpu tests/test_gpu_kernels.py -k "attention or attn" -x || exit 1
for r in 1 2; do
  ENDOSSL_LIB=$OLD run abo_$r 120 python scripts/attn_bench.py --rounds 3 --iters 10 || exit 1
  run abn_$r 120 python scripts/attn_bench.py --rounds 3 --iters 10 || exit 1
done
ENDOSSL_LIB=$OLD run aso 120 python scripts/attn_bench.py --s1 --rounds 3 --iters 5 || exit 1
run asn 120 python scripts/attn_bench.py --s1 --rounds 3 --iters 5 || exit 1
for r in 1 2; do
  ENDOSSL_LIB=$OLD run f1o_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  run f1n_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
done
exit 0
