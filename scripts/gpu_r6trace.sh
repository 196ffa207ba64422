#!/bin/bash
# round 6: kernel traces of the F1 bench and the N = 8 shard; per-step kernel table of steps 3..5 of each
# (scripts/trace_steps.py), to see which kernels -- torch fills included -- run inside step()
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
rm -rf "$OUT/prof" "$OUT/profsh"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit 1
python3 scripts/trace_steps.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" 3 3 400 > "$OUT/f1_steps.txt" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/profsh" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/profsh.log" 2>&1 || exit 1
python3 scripts/trace_steps.py "$(find "$OUT/profsh" -name '*kernel_trace.csv' | head -1)" 5 4 400 > "$OUT/shard_steps.txt" || exit 1
head -3 "$OUT/f1_steps.txt" "$OUT/shard_steps.txt"; grep -i fill "$OUT/f1_steps.txt" "$OUT/shard_steps.txt"; exit 0
