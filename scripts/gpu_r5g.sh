#!/bin/bash
# round 5: F1 / C1 with the grouped weight-gradient launch's CU share (Engine.LAYER_TN_SHARE) around the default
# 0.375, same box, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
arm() {  # arm <name> <share> <bench args...>
  local name=$1 sh=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.vit as v; v.Engine.LAYER_TN_SHARE=$sh; import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm f1s375_$r 0.375 --steps 100 --warmup 5 || exit 1
  arm f1s4375_$r 0.4375 --steps 100 --warmup 5 || exit 1
  arm f1s3125_$r 0.3125 --steps 100 --warmup 5 || exit 1
  arm c1s375_$r 0.375 --workload c1 --steps 10 --warmup 3 || exit 1
  arm c1s4375_$r 0.4375 --workload c1 --steps 10 --warmup 3 || exit 1
done
