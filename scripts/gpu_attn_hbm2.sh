#!/bin/bash
# HBM bytes (FETCH_SIZE / WRITE_SIZE) of the F1 attention kernels after the whole-row output stores and the
# seven-wave forward; one counter per pass
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/attn_bench.py --rounds 1 --iters 2"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/attnhbm2_$i" -o run --output-format csv -- $B > "$OUT/attnhbm2_$i.log" 2>&1
  rc=$?; echo "hbm pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
