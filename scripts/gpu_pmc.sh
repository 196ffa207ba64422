#!/bin/bash
# PMC passes (one counter group per pass; never combined with tracing) over the GEMM microbench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants ${VARIANTS:-0} --rounds 1 --iters 2"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/pmc$i" -o run --output-format csv -- $B > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/pmc$i.log"; break; }
done
exit 0
