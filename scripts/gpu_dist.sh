#!/bin/bash
# GPU pass for the overlapped all-reduce: the 2-rank gloo test on cuda:0, then the step tests.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_dist.py > gpurun_out/dist.log 2>&1; rc=$?
echo "dist rc=$rc"; tail -15 gpurun_out/dist.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 $PT tests/test_gpu_step.py tests/test_gpu_comatch.py > gpurun_out/s.log 2>&1; rc=$?
echo "step rc=$rc"; tail -5 gpurun_out/s.log
exit $rc
