#!/bin/bash
# FCUDown kernels: HEAD library vs working tree (time + bit identity), conformer tests, S1 A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
OLD="$GRAFT_REPO_ROOT/build/ab/HEAD/libendossl_hip.so"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1) $(grep -v amdgpu.ids "$OUT/$name.log" | tail -2 | tr '\n' ' ' | cut -c1-250)"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
ENDOSSL_LIB=$OLD run fo 120 python scripts/fcu_bench.py old || exit 1
run fn 120 python scripts/fcu_bench.py new old || exit 1
run tc 400 $PT -m gpu tests/test_gpu_conformer.py -x || exit 1
for r in 1 2; do
  ENDOSSL_LIB=$OLD run s1o_$r 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
  run s1n_$r 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
done
exit 0
