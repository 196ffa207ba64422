#!/bin/bash
# round 5: the conv weight pack with coalesced stores (LDS-tiled transpose for wt): pack / conformer / resnet
# tests, then P0 and S1, HEAD's library (A) vs this tree's (B), same box, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "pack" > "$OUT/tv.log" 2>&1; rc=$?; tail -1 "$OUT/tv.log"; [ $rc -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resnet.py tests/test_gpu_conformer.py > "$OUT/tv2.log" 2>&1; rc=$?; tail -1 "$OUT/tv2.log"; [ $rc -ne 0 ] && exit 1
R=3 LIM=200 BARGS="--workload p0 --steps 100 --warmup 10" bash scripts/gpu_ab_lib.sh || exit 1
R=2 LIM=240 BARGS="--workload s1 --steps 5 --warmup 2" bash scripts/gpu_ab_lib.sh
