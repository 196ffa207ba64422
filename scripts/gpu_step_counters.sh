#!/bin/bash
# Step-level counters of the F1 bench step (north_star: "rocprof HBM GB/s and MFMA utilisation"): one rocprofv3
# --pmc pass per counter set over bench.py (2 timed steps), each with the kernel trace (durations), then
# scripts/step_counters.py -> profiles/<TAG>_step_counters.{md,json}.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
TAG=${TAG:-r04}
rm -rf "$OUT"/scnt[0-9]*
i=0
for C in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d "$OUT/scnt$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/scnt$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -3 "$OUT/scnt$i.log"; exit 1; }
done
python3 scripts/step_counters.py "$OUT" "$TAG" && cat "profiles/${TAG}_step_counters.md"
