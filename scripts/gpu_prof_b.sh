#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py at a given per-GPU batch (BATCH, default 64) -> gpurun_out/prof_<TAG>
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-b${BATCH:-64}}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --batch ${BATCH:-64} ${EXTRA} > "gpurun_out/prof_$TAG.log" 2>&1
echo "prof $TAG rc=$?"
