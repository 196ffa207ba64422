#!/bin/bash
# round 5: the N = 8 shard with the small-shard grouped weight-gradient launch every GROUP_LAYERS blocks (Engine,
# default 6) at 6 / 8 / 9 / 12 (4 / 3 / 2 / 1: 5.33 / 5.36 / 5.50 / 6.57 vs 5.21 ms), same box, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
arm() {  # arm <name> <group layers> <bench args...>
  local name=$1 gl=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.vit as v; v.Engine.GROUP_LAYERS=$gl; import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  for gl in 6 8 9 12; do
    arm sh_gl${gl}_$r $gl --batch 8 --steps 50 --warmup 10 || exit 1
  done
done
