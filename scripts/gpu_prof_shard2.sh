#!/bin/bash
# kernel trace of the N = 8 per-rank shard step (B = 8, mu = 7 on one GPU)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_shard" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/prof_shard.log" 2>&1; rc=$?
echo "rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$OUT/prof_shard.log"; find "$OUT/prof_shard" -name "*kernel_trace.csv" | head -2
exit $rc
