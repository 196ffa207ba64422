#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1) $(tail -1 "$OUT/$name.log" | cut -c1-120)"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run tst 300 $PT -m gpu tests/test_gpu_conformer.py -k "stem or conv2d_fwd_bwd" -x || exit 1
run sb 200 python scripts/stem_bench.py || exit 1
grep -v amdgpu.ids "$OUT/sb.log"
for r in 1 2; do
  ENDOSSL_STEM_KERNELS=0 run p0g_$r 200 python bench.py --workload p0 --steps 20 --warmup 5 || exit 1
  run p0s_$r 200 python bench.py --workload p0 --steps 20 --warmup 5 || exit 1
done
run s1s 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
exit 0
