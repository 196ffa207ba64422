#!/bin/bash
# HBM bytes per launch of the attention backward at the F1 shape (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction of
# MI355X_MICROARCH.md), one counter per pass over scripts/attn_bench.py: two-pass (3) vs single pass (4)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for C in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/ph$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/attn_bench.py" --no-fwd --bwd 3,4 --rounds 1 --iters 2 > "$OUT/ph$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/ph$i.log"; exit 1; }
done
python3 scripts/pmc_table.py "$OUT"/ph1 "$OUT"/ph2 > "$OUT/attn_hbm.md"; grep -i "attn\|kernel" "$OUT/attn_hbm.md"
timeout -k 10 200 python -u scripts/attn_bench.py --rounds 5 --no-fwd --bwd 3,4 > "$OUT/abench.log" 2>&1; echo "bench rc=$?"; tail -1 "$OUT/abench.log"
exit 0
