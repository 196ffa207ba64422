#!/bin/bash
# Conformer / SemiFormer GPU tests, then the S1 bench line (and, with AB_ENV set, the same line again
# with $AB_ENV exported: a same-box A/B).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_conformer.py > gpurun_out/cf.log 2>&1; rc=$?
echo "cf rc=$rc"; tail -3 gpurun_out/cf.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload s1 --steps 5 --warmup 2 > gpurun_out/s1.log 2>&1; rc=$?
  echo "s1 rc=$rc"; tail -1 gpurun_out/s1.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
  [ -n "$AB_ENV" ] || exit 0
  env $AB_ENV timeout -k 10 300 python bench.py --workload s1 --steps 5 --warmup 2 > gpurun_out/s1_ab.log 2>&1; rc=$?
  echo "s1 [$AB_ENV] rc=$rc"; tail -1 gpurun_out/s1_ab.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
