#!/bin/bash
# SQ / LDS / L2 counters of one NT GEMM shape at the default kernel choice (one pass per counter set).
# usage: ONLY=qkv_fwd bash scripts/gpu_pmc_nt.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants=${NTV:--1} --rounds 1 --iters 2 --only ${ONLY:-qkv_fwd} --tn-variants 0 --tn-blocks auto"
i=0
rm -rf "$OUT"/sq[0-9]*
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/sq$i" -o run --output-format csv -- $B > "$OUT/sq$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/sq$i.log"; break; }
done
exit 0
