#!/bin/bash
# CoMatch + FixMatch GPU tests, then the C1 and F1 bench lines.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_comatch.py tests/test_gpu_step.py tests/test_gpu_kernels.py > gpurun_out/c.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/c.log
[ $rc -eq 0 ] || exit $rc
for w in c1 f1; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$w.log 2>&1; rc=$?
  echo "$w rc=$rc"; tail -1 gpurun_out/b_$w.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
