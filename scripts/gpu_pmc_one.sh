#!/bin/bash
# PMC passes (one counter group per pass, no tracing) over ONE GEMM shape of scripts/gemm_bench.py.
# usage: ONLY=fc1_fwd VARIANTS=-1 bash scripts/gpu_pmc_one.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants=${VARIANTS:--1} --rounds 1 --iters 2 --only ${ONLY:-fc1_fwd} --tn-blocks 1536"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_EA0_WRREQ_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/sq$i" -o run --output-format csv -- $B > "$OUT/sq$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/sq$i.log"; break; }
done
exit 0
