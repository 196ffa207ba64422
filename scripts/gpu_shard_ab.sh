#!/bin/bash
# N=8 / N=4 per-rank shard: the 64-row tiles (default) vs ENDOSSL_GEMM_VARIANT=-3 (the previous rules), and hipGraph
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --steps 20 --warmup 5 --batch $1 --no-cpu-baseline $3 > gpurun_out/sh.log 2>&1 || exit 0
  echo "B=$1 $2 $3: $(grep '^{' gpurun_out/sh.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"; }
for r in 1 2; do
  run 8 new ""
  ENDOSSL_SMALL_TILE=0 run 8 old ""
  run 8 new "--graph on"
  run 16 new ""
  ENDOSSL_SMALL_TILE=0 run 16 old ""
done
