#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT -m gpu -x tests/test_gpu_kernels.py -k attention > "$OUT/ka.log" 2>&1; rc=$?; echo "ka rc=$rc"; tail -2 "$OUT/ka.log"
[ $rc -le 1 ] || exit 0
timeout -k 10 200 python scripts/attn_bench.py --rounds 5 --iters 10 > "$OUT/attn.log" 2>&1; echo "attn rc=$?"; grep -v amdgpu "$OUT/attn.log"
for r in 1 2; do
  for v in 1 2 3; do
    ENDOSSL_ATTN_BWD_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/abv_$v.log" 2>&1 || exit 0
    echo "attn bwd variant $v: $(grep '^{' "$OUT/abv_$v.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
for r in 1 2; do
  for gw in auto 0; do
    ENDOSSL_GROUP_WGRAD=$gw timeout -k 10 200 python bench.py --steps 20 --warmup 5 --batch 8 --no-cpu-baseline > "$OUT/sh_$gw.log" 2>&1 || exit 0
    echo "shard B=8 group=$gw: $(grep '^{' "$OUT/sh_$gw.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
exit 0
