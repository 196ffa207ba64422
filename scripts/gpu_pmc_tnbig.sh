#!/bin/bash
# SQ / LDS / cache counters of the weight-gradient GEMM variants at the fc1 wgrad shape (one pass per counter set).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants 5 --rounds 1 --iters 2 --only ${ONLY:-fc1_wgrad} --tn-variants ${TNV:-0,7} --tn-blocks auto"
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/sq$i" -o run --output-format csv -- $B > "$OUT/sq$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/sq$i.log"; break; }
done
exit 0
