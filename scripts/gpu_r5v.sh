#!/bin/bash
# round 5: the few-column dense forward (a classifier head: one wave per output): dense / head / trainer tests,
# then P0, HEAD's library (A) vs this tree's (B), same box, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_comatch.py tests/test_gpu_resnet.py tests/test_gpu_conformer.py > "$OUT/tv.log" 2>&1; rc=$?; tail -1 "$OUT/tv.log"; [ $rc -ne 0 ] && exit 1
R=3 LIM=200 BARGS="--workload p0 --steps 100 --warmup 10" bash scripts/gpu_ab_lib.sh || exit 1
R=2 LIM=200 BARGS="--workload c1 --steps 10 --warmup 3" bash scripts/gpu_ab_lib.sh
