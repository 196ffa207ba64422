#!/bin/bash
# round 5: kernel trace of the S1 step on this tree (rocprofv3 --kernel-trace --stats)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
rm -rf "$OUT/s1prof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/s1prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload s1 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/s1prof.log" 2>&1; echo "s1prof rc=$?"
