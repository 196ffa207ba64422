#!/bin/bash
# SQ counters of NT GEMM shapes at the default kernel choice, one pass per counter set; + the counter list
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1; echo "list rc=$?"
for SH in ${SHAPES:-qkv_fwd fc1_fwd_weak fc2_fwd}; do
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants=${NTV:--1} --rounds 1 --iters 2 --only $SH --tn-variants 0 --tn-blocks auto"
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
         "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/pmc_$SH/sq$i" -o run --output-format csv -- $B > "$OUT/pmc_$SH.sq$i.log" 2>&1
  rc=$?; echo "$SH pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/pmc_$SH.sq$i.log"; exit 0; }
done
python3 scripts/pmc_ratios.py "$OUT/pmc_$SH"/sq*
done
exit 0
