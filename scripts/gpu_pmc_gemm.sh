#!/bin/bash
# SQ counter passes (two groups, no tracing) over one GEMM microbenchmark shape.
# usage: ONLY=fc1_wgrad bash scripts/gpu_pmc_gemm.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants=-1 --rounds 1 --iters 2 --tn-variants 0 --tn-blocks 1536 --only ${ONLY:-fc1_fwd}"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/gpmc_${ONLY:-fc1_fwd}_$i" -o run --output-format csv -- $B > "$OUT/gpmc$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/gpmc$i.log"; exit $rc; }
done
exit 0
