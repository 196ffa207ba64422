#!/bin/bash
# SQ counters of the grouped weight-gradient launch (the bench's roofline kernel) in the F1 step: one --pmc pass
# per counter set over bench.py (2 timed steps), per-kernel means -> gpurun_out/pmc_wgrad.md
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/pw$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pw$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/pw$i.log"; exit 1; }
done
python3 scripts/pmc_table.py "$OUT"/pw1 "$OUT"/pw2 > "$OUT/pmc_wgrad.md"; grep -i "kernel\|tn_big_grouped\|splitk" "$OUT/pmc_wgrad.md" | head -8
exit 0
