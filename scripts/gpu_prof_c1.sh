#!/bin/bash
# rocprofv3 summaries of C1 (default streams) and the hipGraph form of the N=8 shard
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -1)"; return $rc; }
run g8on 200 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline --graph on || exit 1
run g8off 200 python bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run c1prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/c1prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c1 --steps 3 --warmup 2 || exit 1
exit 0
