#!/bin/bash
# SQ counter passes over the attention microbenchmark (one counter group per pass, no tracing)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/attn_bench.py --rounds 1 --iters 2"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/attnpmc3_$i" -o run --output-format csv -- $B > "$OUT/attnpmc3_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/attnpmc3_$i.log"; exit $rc; }
done
exit 0
