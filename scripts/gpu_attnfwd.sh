#!/bin/bash
# attention forward with the scale folded into a packed fma: tests, microbench, F1 / S1 step
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run ta 400 $PT -m gpu tests/test_gpu_kernels.py tests/test_gpu_step.py tests/test_gpu_blocks.py tests/test_gpu_parity.py -x || exit 1
run ab 120 python scripts/attn_bench.py --rounds 3 --iters 10 || exit 1
run f1 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run s1 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
run tcf 300 $PT -m gpu tests/test_gpu_conformer.py -x || exit 1
exit 0
