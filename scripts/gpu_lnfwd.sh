#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/ln_bench.py > "$OUT/lnb.log" 2>&1 || { tail -5 "$OUT/lnb.log"; exit 1; }
grep -v amdgpu.ids "$OUT/lnb.log"
AV="es_set_ln_fwd_grid=0 es_set_ln_fwd_grid=${G:-2048}" bash scripts/gpu_ab_knobs.sh
