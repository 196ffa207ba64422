#!/bin/bash
# round 5: F1 / C1 with the LayerNorm backward's workgroup count (vit.LN_BWD_BLOCKS, default 1024) at 1024 / 2048 /
# 512, same box, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
arm() {  # arm <name> <blocks> <bench args...>
  local name=$1 nb=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.vit as v; v.LN_BWD_BLOCKS=$nb; import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  for nb in 1024 2048 512; do
    arm f1_lnb${nb}_$r $nb --steps 100 --warmup 5 || exit 1
  done
  for nb in 1024 2048; do
    arm c1_lnb${nb}_$r $nb --workload c1 --steps 10 --warmup 3 || exit 1
  done
done
