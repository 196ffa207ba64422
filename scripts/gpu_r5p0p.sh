#!/bin/bash
# round 5: kernel trace of the graph-replayed P0 step (bf16 maps) on this tree
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
rm -rf "$OUT/p0prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p0prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload p0 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/p0prof.log" 2>&1; echo "p0prof rc=$?"
