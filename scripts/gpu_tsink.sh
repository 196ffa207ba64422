#!/bin/bash
# token-buffer gradient sink: conformer tests, S1 same-box A/B against HEAD (its library + python package)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1) $(grep -o '"final_loss": [0-9.e-]*' "$OUT/$name.log" | head -1) $(grep -v amdgpu.ids "$OUT/$name.log" | tail -1 | cut -c1-100)"; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run tc 500 $PT -m gpu tests/test_gpu_conformer.py tests/test_gpu_fullsize.py tests/test_gpu_convs.py -x || exit 1
for r in 1 2; do
  ENDOSSL_TOKEN_SINK=0 run s1o_$r 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
  run s1n_$r 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
done
exit 0
