#!/bin/bash
# bf16 CNN maps: kernel bit-exactness, model / trainer / per-conv / full-size S1 tests, then the S1 bench
# with bf16 maps and with ENDOSSL_MAP_BF16=0 (same box).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT -x tests/test_gpu_conformer.py -k "bf16_maps" > gpurun_out/mk.log 2>&1; rc=$?
echo "maps kernels rc=$rc"; tail -3 gpurun_out/mk.log
[ $rc -eq 0 ] || exit 0
timeout -k 10 500 $PT tests/test_gpu_conformer.py tests/test_gpu_convs.py tests/test_gpu_fullsize.py -k "not bf16_maps and not c1" > gpurun_out/mm.log 2>&1; rc=$?
echo "model rc=$rc"; tail -8 gpurun_out/mm.log
[ $rc -le 1 ] || exit 0
for r in 1 2; do
  for mb in 1 0; do
    ENDOSSL_MAP_BF16=$mb timeout -k 10 300 python bench.py --workload s1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/s1_$mb.log 2>&1 || exit 0
    echo "s1 maps_bf16=$mb: $(grep '^{' gpurun_out/s1_$mb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
