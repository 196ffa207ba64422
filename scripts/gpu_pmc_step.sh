#!/bin/bash
# HBM bytes of a whole F1 step: FETCH_SIZE and WRITE_SIZE passes (one counter set per run) over
# bench.py; summed per kernel by scripts/pmc_step_bytes.py.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
rm -rf "$OUT"/pstep[0-9]*
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/pstep$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${EXTRA} > "$OUT/pstep$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/pstep$i.log"; break; }
done
exit 0
