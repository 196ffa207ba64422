#!/bin/bash
# rocprofv3 kernel trace of the per-rank F1 shard at N=8 (B=8, mu=7) on one GPU, and its bench line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/shard.log" 2>&1 || exit 1
tail -1 "$OUT/shard.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("shard", d["ms_per_step"], d["value"])'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/profsh" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/profsh.log" 2>&1; echo "prof rc=$?"
exit 0
