#!/bin/bash
# SQ counters of the attention backward kernels at the F1 shape (two-pass dq2 + dkv2 vs the single pass), one
# pass per counter set, no tracing
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pa$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/attn_bench.py" --no-fwd --bwd ${BWD:-3,4} --rounds 1 --iters 2 > "$OUT/pa$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/pa$i.log"; break; }
done
python3 scripts/pmc_table.py "$OUT"/pa1 "$OUT"/pa2 "$OUT"/pa3 > "$OUT/pmc_attn.md"; cat "$OUT/pmc_attn.md"
exit 0
