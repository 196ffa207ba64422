#!/bin/bash
# the weak / train forwards' launches interleaved block by block (Engine.forward_pair) vs one after the
# other: tests, the N = 8 shard (B = 8) and F1, same box
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run ts 400 $PT -m gpu tests/test_gpu_step.py -x || exit 1
for r in 1 2; do
  ENDOSSL_FWD_INTERLEAVE=0 run b8o_$r 200 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  run b8n_$r 200 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
for r in 1 2; do
  ENDOSSL_FWD_INTERLEAVE=0 run b16o_$r 200 python bench.py --batch 16 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  run b16n_$r 200 python bench.py --batch 16 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
for r in 1 2; do
  ENDOSSL_FWD_INTERLEAVE=0 run f1o_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  run f1n_$r 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
done
exit 0
