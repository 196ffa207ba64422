#!/bin/bash
# pipelined attention forward: kernel tests, isolated timing at the F1 head batch, then live F1 A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention_fwd" > "$OUT/tap.log" 2>&1; rc=$?; tail -2 "$OUT/tap.log"; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u scripts/attn_bench.py --fwd 7,8,8g0,8g768,8g1024,9,9g0,9g768 --bwd 4 --rounds 5 > "$OUT/abp.log" 2>&1 || { tail -5 "$OUT/abp.log"; exit 1; }
grep -v amdgpu.ids "$OUT/abp.log"
AV="es_set_attn_variant=7 es_set_attn_variant=8 es_set_attn_variant=9 es_set_attn_variant=8,es_set_attn_fwd_grid=768" bash scripts/gpu_ab_knobs.sh
