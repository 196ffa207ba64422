#!/bin/bash
# kernel trace of the C1 step (CoMatch, B=64, mu=7, Q=65,536)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/c1prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c1 --steps 4 --warmup 2 > "$OUT/c1prof.log" 2>&1; rc=$?
echo "rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$OUT/c1prof.log"
exit $rc
