#!/bin/bash
# S1: 256x256 (one workgroup per CU, 128-KiB LDS) vs 256x128 two-per-CU tiles for the transformer GEMMs beside the CNN branch
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for r in 1 2; do
  for v in "es_set_gemm_wide_tile=1" "es_set_gemm_wide_tile=0" "es_set_tn_variant=0" "es_set_gemm_wide_tile=0,es_set_tn_variant=0"; do
    i=$((i+1))
    timeout -k 10 300 python -u scripts/s1_knob_ab.py $(echo $v | tr "," " ") > "$OUT/abw_$i.log" 2>&1 || { tail -3 "$OUT/abw_$i.log"; exit 1; }
    echo "$v $(tail -1 $OUT/abw_$i.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
  done
done
