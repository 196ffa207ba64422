#!/bin/bash
# Teacher-forced per-block parity at F1 (tests/test_gpu_blocks.py), then the full GPU pass.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 400 python -u -m pytest -q -rf -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_blocks.py > "$OUT/blocks.log" 2>&1; rc=$?
echo "blocks rc=$rc"; tail -5 "$OUT/blocks.log"
[ $rc -le 1 ] || exit 0
PROFILE=0 bash scripts/gpu_check.sh
