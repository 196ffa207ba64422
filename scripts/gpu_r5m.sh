#!/bin/bash
# round 5: long-sequence attention changes -- outputs of the tree's build against the previous build (libA) bit
# for bit at the S1 shape, interleaved timing of both builds (scripts/attn_bench.py --s1), then the attention
# GPU tests and an S1 A/B (scripts/gpu_ab_lib.sh)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
A=$PWD/endoscopy-image-classification_amd/csrc/build/ab/libA.so
ENDOSSL_LIB=$A timeout -k 10 200 python3 scripts/attn_bench.py --s1 --rounds 1 --iters 2 --bwd 0,3 --save /tmp/attn_a.pt > "$OUT/ab0.log" 2>&1 || { tail -3 "$OUT/ab0.log"; exit 1; }
timeout -k 10 200 python3 scripts/attn_bench.py --s1 --rounds 1 --iters 2 --bwd 0,3 --compare /tmp/attn_a.pt > "$OUT/ab1.log" 2>&1 || { tail -3 "$OUT/ab1.log"; exit 1; }
grep "bit-identical" "$OUT/ab1.log"
for r in 1 2 3; do
  ENDOSSL_LIB=$A timeout -k 10 200 python3 scripts/attn_bench.py --s1 --rounds 3 --iters 10 --bwd 3 > "$OUT/aa$r.log" 2>&1 || exit 1
  timeout -k 10 200 python3 scripts/attn_bench.py --s1 --rounds 3 --iters 10 --bwd 3 > "$OUT/ab$r.log" 2>&1 || exit 1
  echo "round $r A $(tail -1 $OUT/aa$r.log | cut -c1-200)"
  echo "round $r B $(tail -1 $OUT/ab$r.log | cut -c1-200)"
done
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_s1_blocks.py tests/test_gpu_kernels.py -k "attn or s1" > "$OUT/ta.log" 2>&1; rc=$?; tail -2 "$OUT/ta.log"; [ $rc -ne 0 ] && exit 1
R=3 LIM=200 BARGS="--workload s1 --steps 5 --warmup 2" bash scripts/gpu_ab_lib.sh || exit 1
exit 0
