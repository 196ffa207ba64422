#!/bin/bash
# 128x384 whole-row NT tiles (variants 16 / 18): GEMM tests, isolated sweep at F1 and the N = 8 shard
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm_nt" > "$OUT/t16.log" 2>&1; rc=$?; tail -2 "$OUT/t16.log"; [ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py --variants=-1,16,18,10,0 --rounds 5 > "$OUT/gb16.log" 2>&1 || { tail -5 "$OUT/gb16.log"; exit 1; }
timeout -k 10 300 python -u scripts/gemm_bench.py --variants=-1,16,18,11,0 --rounds 5 --shard 8 > "$OUT/gb16s.log" 2>&1 || { tail -5 "$OUT/gb16s.log"; exit 1; }
grep -v "^#" "$OUT/gb16.log" | head -40
exit 0
