#!/bin/bash
# round 5: SQ counters of the attention kernels (scripts/attn_bench.py), one --pmc pass per counter set ->
# gpurun_out/pmc_attn_$TAG.md.  TAG=s1 (default): the S1 long-sequence kernels; TAG=f1 ARGS="--rounds 1 --iters 2
# --bwd 4": the F1 shape with the single-pass backward
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
TAG=${TAG:-s1}; ARGS=${ARGS:---s1 --rounds 1 --iters 2 --bwd 0}
rm -rf "$OUT"/pa_${TAG}_[0-9]
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
         "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pa_${TAG}_$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/attn_bench.py" $ARGS > "$OUT/pa_${TAG}_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/pa_${TAG}_$i.log"; break; }
done
python3 scripts/pmc_table.py "$OUT"/pa_${TAG}_[0-9] > "$OUT/pmc_attn_$TAG.md"; grep -i "attn" "$OUT/pmc_attn_$TAG.md" | head -20
exit 0
