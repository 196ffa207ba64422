#!/bin/bash
# SQ counters of the panel K=384 GEMM (variant 30) against the default tiles at the F1 shapes (one pass
# per counter set, no tracing)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pc$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/gemm_bench.py" --variants=${VARIANTS:--1,30} --rounds 1 --iters 3 --only ${ONLY:-qkv_fwd,fc2_dgrad} > "$OUT/pc$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/pc$i.log"; break; }
done
python3 scripts/pmc_table.py "$OUT"/pc1 "$OUT"/pc2 > "$OUT/pmc_panel.md"; cat "$OUT/pmc_panel.md"
exit 0
