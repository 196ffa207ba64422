#!/bin/bash
# specialised stem conv kernels: tests, then S1 / P0 same-box A/B (es_set_stem_kernels via ENDOSSL_STEM_KERNELS)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1) $(tail -1 "$OUT/$name.log" | cut -c1-120)"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run tst 300 $PT -m gpu tests/test_gpu_conformer.py -k "stem or conv2d_fwd_bwd" -x || exit 1
run tres 300 $PT -m gpu tests/test_gpu_resnet.py tests/test_gpu_convs.py -x || exit 1
for r in 1 2; do
  ENDOSSL_STEM_KERNELS=0 run s1g_$r 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
  run s1s_$r 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
done
ENDOSSL_STEM_KERNELS=0 run p0g 200 python bench.py --workload p0 --steps 10 --warmup 3 || exit 1
run p0s 200 python bench.py --workload p0 --steps 10 --warmup 3 || exit 1
exit 0
