#!/bin/bash
# SQ / TA counter passes (one group per pass, no tracing) over selected GEMM shapes:
# where do the waves' cycles go (parked on waits, issue-stalled, active VALU / MFMA / LDS)?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1; echo "list rc=$?"
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants ${VARIANTS:-5,1} --rounds 1 --iters 2 --only ${ONLY:-fc1_fwd,fc2_fwd,fc1_dgrad,fc2_wgrad}"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
         "TA_TA_BUSY_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d "$OUT/sq$i" -o run --output-format csv -- $B > "$OUT/sq$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/sq$i.log"; [ $rc -gt 1 ] && [ $rc -ne 2 ] && break; }
done
exit 0
