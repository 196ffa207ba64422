#!/bin/bash
# SQ counters of the weight-stationary NT GEMM (variant 12) in scripts/ws_bench.py, per probe (ENDOSSL_WS_PROBE,
# measurement builds only): PROBES="0 4" ONLY=qkv_fwd -> gpurun_out/pmc_ws_p<probe>.md
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
for pr in ${PROBES:-0 4}; do
  i=0
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    ENDOSSL_WS_PROBE=$pr timeout -s KILL 100 rocprofv3 --pmc $C -d "$OUT/pws${pr}_$i" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/scripts/ws_bench.py" --rounds 1 --iters 3 --only ${ONLY:-qkv_fwd} > "$OUT/pws${pr}_$i.log" 2>&1
    rc=$?; echo "probe $pr pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -3 "$OUT/pws${pr}_$i.log"; exit 1; }
  done
  python3 scripts/pmc_table.py "$OUT"/pws${pr}_1 "$OUT"/pws${pr}_2 > "$OUT/pmc_ws_p$pr.md"
done
exit 0
